"""Keyswitch time (lincomb + digit pass + GEMM, kernel-stamped timers at profiling level
2) of OR levels by fan-in, for A/B runs of library variants (FHEREGEX_LIB=...): G
independent threshold ORs of F booleans each (Context.or_each: one keyswitch + one
blind-rotation launch), median over R repetitions.  The match's OR levels are such
levels (/abc/ x 256: 16 ORs of 16, then 1 of 16).
Usage: python3 tools/ks_fanin_probe.py [reps]"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
import fheregex as F  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
    blob = f.read()
ctx = F.Context(0)
ctx.load_client_key(blob)
ctx.gen_server_key(42)
hs = ctx.upload_bool(ctx.encrypt_blocks([0] * 63 + [1], seed=3))
out = {}
for G, fan in [(1, 16), (16, 16), (254, 6), (512, 2)]:
    groups = [[hs[(g * fan + i) % len(hs)] for i in range(fan)] for g in range(G)]
    for h in ctx.or_each(groups):  # warm-up
        ctx.release(h)
    ks = []
    for _ in range(reps):
        t0 = ctx.device_timers()
        ctx.set_profiling(2)
        res = ctx.or_each(groups)
        ctx.set_profiling(0)
        t1 = ctx.device_timers()
        ks.append((t1["ks_ms"] - t0["ks_ms"]) * 1e3)
        for h in res:
            ctx.release(h)
    out[f"{G}x{fan}"] = round(statistics.median(ks), 1)
print(os.path.basename(os.environ.get("FHEREGEX_LIB", "libfheregex.so")), "ks_us", out, flush=True)
