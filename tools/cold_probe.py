"""Cold-call host cost split: first has_match's host_ms (record + lower + compile + uploads)
against the host-only schedule (record + lower + build_schedule, fr_schedule_match), per
BASELINE workload.  Usage: python3 tools/cold_probe.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402
from bench import WORKLOADS, make_content  # noqa: E402

with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0)
ctx.load_client_key(blob)
ctx.gen_server_key(42)
for name in ("metric", "config3", "config4", "config5"):
    W = WORKLOADS[name]
    g = W.get("grammar", F.GRAMMAR_REFERENCE)
    ctx.set_grammar(g)
    L = W["chars"]
    hs = ctx.upload_radix(ctx.encrypt_str(make_content(W["content"], L).decode(), seed=3))
    t = time.perf_counter()
    S = F.schedule_match(L, W["pattern"], grammar=g)
    sched_ms = (time.perf_counter() - t) * 1e3 / 2  # schedule_match calls the library twice
    ctx.set_plan_cache(0)
    out, st = ctx.has_match(hs, W["pattern"])
    ctx.download_radix(out)
    out2, st2 = ctx.has_match(hs, W["pattern"])
    ctx.download_radix(out2)
    print(f"{name}: L={L} rotations={len(S.jobs)} host-only schedule {sched_ms:.2f} ms; first call host "
          f"{st.host_ms:.2f} ms, again (cache off) {st2.host_ms:.2f} ms", flush=True)
    for h in list(hs) + [out, out2]:
        ctx.release(h)
    ctx.set_plan_cache(8)
