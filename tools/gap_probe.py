"""Launch gaps of the /abc/ x 256 match with the per-level event timers on or off: run
under `rocprofv3 --kernel-trace` and compare the kernel trace's gaps between dependent
launches.  Usage: python3 tools/gap_probe.py on|off [matches]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402
from bench import make_content  # noqa: E402

prof = {"on": 1, "off": 0, "all": 2}[sys.argv[1]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0)
ctx.load_client_key(blob)
ctx.gen_server_key(42)
hs = ctx.upload_radix(ctx.encrypt_str(make_content("printable", 256).decode(), seed=7))
for _ in range(3):
    o, _ = ctx.has_match(hs, "/abc/")
    ctx.release(o)
ctx.set_profiling(prof)
outs = [ctx.has_match(hs, "/abc/")[0] for _ in range(n)]
print("result", ctx.decrypt_radix(ctx.download_radix(outs[-1])), "profiling", prof, flush=True)
