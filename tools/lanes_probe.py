"""Matches in flight on ONE context (fr_set_lanes) against the serial match: wall time per
/abc/ x 256 match amortised over back-to-back asynchronous matches, for each lane count.
Usage: python3 tools/lanes_probe.py [matches] [lanes...]   (GPU_MAX_HW_QUEUES from the env)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import numpy as np  # noqa: E402

import fheregex as F  # noqa: E402
from bench import make_content  # noqa: E402

nm = int(sys.argv[1]) if len(sys.argv) > 1 else 24
lanes = [int(x) for x in sys.argv[2:]] or [1, 2, 3, 4]
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0)
ctx.load_client_key(blob)
ctx.gen_server_key(42)
hs = np.asarray(ctx.upload_radix(ctx.encrypt_str(make_content("printable", 256).decode(), seed=7)), dtype=np.uint32)
ref = None
out = {}
for L in lanes:
    ctx.set_lanes(L)
    for _ in range(max(L, 2)):  # every lane's plan
        ctx.release(ctx.has_match(hs, "/abc/")[0])
    ctx.download_radix(int(hs[0]))
    best = None
    for rep in range(3):
        t = time.perf_counter()
        outs = [ctx.has_match(hs, "/abc/")[0] for _ in range(nm)]
        w = ctx.download_radix(outs[-1])
        ms = (time.perf_counter() - t) * 1e3 / nm
        best = ms if best is None else min(best, ms)
        words = [ctx.download_radix(o) for o in outs]
        if ref is None:
            ref = words[0]
        assert all(np.array_equal(x, ref) for x in words), L
        for o in outs:
            ctx.release(o)
    out[L] = round(best, 3)
    ctx.set_lanes(1)
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES", "(default)"), "ms per match by lanes", out, flush=True)
