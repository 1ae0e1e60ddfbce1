"""Two (or more) /abc/ x 256 matches in flight: C contexts on one GPU, each with its own
stream and copy of the keys, matches dealt round-robin; wall time per match amortised over
R matches, against the same matches on one context.  Usage: python3 tools/inflight_probe.py [C] [R]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402
from bench import make_content  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2
R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
s = make_content("printable", 256).decode()
ctxs, hss = [], []
for i in range(C):
    c = F.Context(0)
    c.load_client_key(blob)
    c.gen_server_key(42)
    ctxs.append(c)
    hss.append(c.upload_radix(c.encrypt_str(s, seed=7 + i)))
for c, hs in zip(ctxs, hss):
    for _ in range(2):
        c.release(c.has_match(hs, "/abc/")[0])
    c.download_radix(hs[0])


def run(nctx):
    outs = []
    t = time.perf_counter()
    for i in range(R):
        k = i % nctx
        outs.append((k, ctxs[k].has_match(hss[k], "/abc/")[0]))
    res = [ctxs[k].decrypt_radix(ctxs[k].download_radix(o)) for k, o in outs]
    dt = (time.perf_counter() - t) * 1e3 / R
    for k, o in outs:
        ctxs[k].release(o)
    assert res == [1] * R
    return dt


for _ in range(2):
    one = run(1)
    many = run(C)
    print(f"one context {one:.3f} ms/match; {C} contexts in flight {many:.3f} ms/match ({one / many:.2f}x)", flush=True)
