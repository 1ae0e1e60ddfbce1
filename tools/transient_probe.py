"""Does a launch run slower right after the chip was lightly loaded?

In the timed region of the bench the 512-bootstrap pair launch (level 1 of `/abc/` x 256) takes
~2.75 ms; back to back it takes ~2.43 ms (tools/power_probe.py).  This times the same launch
after different predecessors, each pattern repeated, one synchronous `fr_dev_bench_pbs` call per
launch (keyswitch + blind rotation; br_ms is the blind rotation alone):

  steady     512, 512, 512, ...
  match      512, 254, 16, 1, 512, 254, 16, 1, ...   (a match's level sizes)
  idle_Xms   512, sleep X ms, 512, ...

    python tools/transient_probe.py OUT.json
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "fhe-regex_amd"))


def main():
    import numpy as np
    import fheregex as F
    blob = open(os.path.join(ROOT, "tests", "golden", "client_key"), "rb").read()
    ck, _ = F.gen_keys(blob, seed=1, device=0)
    ctx = ck.ctx
    rng = np.random.default_rng(5)
    hs = ctx.encrypt_upload_str("".join(chr(c) for c in rng.integers(0x20, 0x7F, 256)), seed=3)
    sel = {c: [hs[i % len(hs)] for i in range(c)] for c in (1, 16, 254, 512)}
    for c in sel:
        ctx.dev_bench_pbs(sel[c], 3)

    def one(c):
        return ctx.dev_bench_pbs(sel[c], 1)[0]

    out = {}
    reps = 40
    # steady
    xs = [one(512) for _ in range(reps)]
    out["steady_512"] = xs
    # match pattern
    rec = {c: [] for c in (512, 254, 16, 1)}
    for _ in range(reps):
        for c in (512, 254, 16, 1):
            rec[c].append(one(c))
    out["match"] = {str(c): v for c, v in rec.items()}
    # idle gaps
    for gap in (1, 4, 10):
        xs = []
        for _ in range(reps):
            time.sleep(gap / 1e3)
            xs.append(one(512))
        out[f"idle_{gap}ms_512"] = xs
    # a lone bootstrap after idle vs after a heavy launch
    xs, ys = [], []
    for _ in range(reps):
        time.sleep(0.004)
        xs.append(one(1))
        one(512)
        ys.append(one(1))
    out["lone_after_idle"] = xs
    out["lone_after_512"] = ys
    summ = {}
    for k, v in out.items():
        if isinstance(v, dict):
            for c, w in v.items():
                summ[f"{k}_{c}"] = float(np.median(w[2:]))
        else:
            summ[k] = float(np.median(v[2:]))
    out["median_br_ms"] = summ
    with open(sys.argv[1], "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
