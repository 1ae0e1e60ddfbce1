"""Why is the /abc/ match's 512-bootstrap launch slower than the probe's?  One process:
probe launches (dev_bench_pbs, eq-nibble direct jobs) before and after profiled matches
(multi-value jobs), with the per-shape device timers of the matches.
Usage: python3 tools/pair_gap.py"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import numpy as np  # noqa: E402

import fheregex as F  # noqa: E402

with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0, params=F.default_params(k=1, N=2048))
ctx.load_client_key(blob)
ctx.gen_server_key(42)
rng = np.random.default_rng(0)
s = "".join(chr(c) for c in rng.integers(0x20, 0x7F, 256))
s = s[:200] + "abc" + s[203:]
content = ctx.upload_radix(ctx.encrypt_str(s, seed=1))


def probe(handles, n, reps=5):
    hs = [handles[i % len(handles)] for i in range(n)]
    ctx.dev_bench_pbs(hs, 1)
    return round(statistics.median(ctx.dev_bench_pbs(hs, 1)[0] for _ in range(reps)), 4)


bools = ctx.upload_bool(ctx.encrypt_blocks([i % 16 for i in range(64)], seed=3))
print("probe 512 (64 bool inputs):", probe(bools, 512), flush=True)
print("probe 512 (256 content chars):", probe(content, 512), flush=True)
ctx.set_profiling(True)
for _ in range(3):
    ctx.has_match(content, "/abc/")
t0 = ctx.device_timers()
for _ in range(10):
    o, st = ctx.has_match(content, "/abc/")
t1 = ctx.device_timers()
d = {k: t1[k] - t0[k] for k in t1}
print("match: pair avg ms", round(d["pair_br_ms"] / max(1, d["pair_launches"]), 4), "launches", d["pair_launches"],
      "latency avg ms", round(d["lat_br_ms"] / max(1, d["lat_launches"]), 4), flush=True)
ctx.set_profiling(False)
print("probe 512 (256 content chars) after:", probe(content, 512), flush=True)
