"""Keyswitch launch times (dev_bench_pbs total - blind rotation) for A/B runs of
keyswitch settings (FR_KS_* environment variables, device.h): median over R
repetitions at the given batch sizes.  Usage: python3 tools/ks_probe.py [reps] [sizes...]"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
sizes = [int(x) for x in sys.argv[2:]] or [1, 17, 254, 512]
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0)
ctx.load_client_key(blob)
ctx.gen_server_key(42)
hs = ctx.upload_bool(ctx.encrypt_blocks([i % 16 for i in range(64)], seed=3))
out = {}
for cnt in sizes:
    batch = [hs[i % len(hs)] for i in range(cnt)]
    ctx.dev_bench_pbs(batch, 1)
    ks = []
    for _ in range(reps):
        br, tot = ctx.dev_bench_pbs(batch, 1)
        ks.append((tot - br) * 1e3)
    out[cnt] = round(statistics.median(ks), 1)
env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("FR_KS"))
if os.environ.get("FHEREGEX_LIB"):
    env = (env + " lib=" + os.path.basename(os.environ["FHEREGEX_LIB"])).strip()
print(env or "default", "ks_us", out, flush=True)
