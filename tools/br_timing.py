"""Run blind-rotation batches of a few sizes (for the FR_BR_TIMING debug build:
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_timing.so python3 tools/br_timing.py).
FR_RING=fft|rns selects the ring (default: the library default)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402

with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ring = {"fft": F.RING_FFT, "rns": F.RING_RNS}.get(os.environ.get("FR_RING", ""))
ctx = F.Context(0, params=F.default_params(ring=ring))
ctx.load_client_key(blob)
ctx.gen_server_key(42)
blocks = ctx.encrypt_blocks([i % 16 for i in range(64)], seed=3)
hs = ctx.upload_bool(blocks)
for cnt in [int(x) for x in (sys.argv[1:] or ["1", "256", "1024"])]:
    ctx.dev_bench_pbs([hs[i % len(hs)] for i in range(cnt)], 1)  # warm-up
    br, tot = ctx.dev_bench_pbs([hs[i % len(hs)] for i in range(cnt)], 1)
    print(f"count={cnt} br_ms={br:.3f} total_ms={tot:.3f}", flush=True)
