"""Wall-clock match time of /abc/ on 256 printable chars with the per-level event
timers (profiling mode, bench.py's timed region) off and on, interleaved; median
over R rounds.  Usage: python3 tools/match_probe.py [rounds]"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402
from bench import make_content  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 15
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0)
ctx.load_client_key(blob)
ctx.gen_server_key(42)
hs = ctx.upload_radix(ctx.encrypt_str(make_content("printable", 256).decode(), seed=7))
for _ in range(3):
    o, _ = ctx.has_match(hs, "/abc/")
    ctx.release(o)
res = {False: [], True: []}
for _ in range(rounds):
    for prof in (False, True):
        ctx.set_profiling(prof)
        t0 = time.perf_counter()
        outs = [ctx.has_match(hs, "/abc/")[0] for _ in range(5)]
        ctx.download_radix(outs[-1])  # synchronises the stream
        res[prof].append((time.perf_counter() - t0) / 5 * 1e3)
        for o in outs:
            ctx.release(o)
        ctx.set_profiling(False)
print(os.path.basename(os.environ.get("FHEREGEX_LIB", "libfheregex.so")), "match_ms timers_off %.3f timers_on %.3f" % (statistics.median(res[False]), statistics.median(res[True])), flush=True)
