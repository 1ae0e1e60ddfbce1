"""Wall-clock /abc/ x 256 match time (10 back-to-back asynchronous matches, one
synchronise) for A/B runs of library variants (FHEREGEX_LIB=...): median over R rounds.
Usage: python3 tools/match_ab.py [rounds]"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402
from bench import make_content  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
k, N = (2, 1024) if os.environ.get("FR_PARAMS") == "k2n1024" else (1, 2048)  # as lat_probe.py
ctx = F.Context(0, params=F.default_params(k=k, N=N))
ctx.load_client_key(blob)
ctx.gen_server_key(42)
hs = ctx.upload_radix(ctx.encrypt_str(make_content("printable", 256).decode(), seed=7))
for _ in range(3):
    o, _ = ctx.has_match(hs, "/abc/")
    ctx.release(o)
ms = []
for _ in range(rounds):
    ctx.download_radix(hs[0])  # synchronise
    t0 = time.perf_counter()
    outs = [ctx.has_match(hs, "/abc/")[0] for _ in range(10)]
    ctx.download_radix(outs[-1])
    ms.append((time.perf_counter() - t0) * 1e3 / 10)
    for o in outs:
        ctx.release(o)
print(os.path.basename(os.environ.get("FHEREGEX_LIB", "libfheregex.so")), "match_ms", round(statistics.median(ms), 4),
      "min", round(min(ms), 4), flush=True)
