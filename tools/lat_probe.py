"""Blind-rotation launch times for A/B runs of library variants (FHEREGEX_LIB=...):
median over R repetitions of dev_bench_pbs at the given batch sizes.
Usage: python3 tools/lat_probe.py [reps] [sizes...]"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
sizes = [int(x) for x in sys.argv[2:]] or [1, 16, 254, 512, 2048]
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
k, N = (2, 1024) if os.environ.get("FR_PARAMS") == "k2n1024" else (1, 2048)
ctx = F.Context(0, params=F.default_params(k=k, N=N))
ctx.load_client_key(blob)
if os.environ.get("FR_LAT_PROBE_HOSTKEY"):  # keys through the host upload path (experiment layouts)
    ctx.set_keygen(F.KEYGEN_HOST)
ctx.gen_server_key(42)
hs = ctx.upload_bool(ctx.encrypt_blocks([i % 16 for i in range(64)], seed=3))
out = {}
for cnt in sizes:
    batch = [hs[i % len(hs)] for i in range(cnt)]
    ctx.dev_bench_pbs(batch, 1)  # warm-up
    out[cnt] = round(statistics.median(ctx.dev_bench_pbs(batch, 1)[0] for _ in range(reps)), 4)
print(os.path.basename(os.environ.get("FHEREGEX_LIB", "libfheregex.so")), out, flush=True)
