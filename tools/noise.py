"""Measure TFHE noise on the GPU path (not a test; writes a JSON summary).

Phases are computed with the fixture client key (host numpy), errors are
phase - expected*Delta on the 2^64 torus (signed), reported as log2 of the
standard deviation and of the max |error|:
  fresh    : fresh encryptions (glwe sigma)
  ks       : after keyswitch to the small key (2048 -> 742)
  ms       : after the modulus switch of the keyswitched LWE to 2N (the phase the blind
             rotation decides on; in torus units, decision threshold Delta/2 = 2^58),
             with the Gaussian failure estimate per bootstrap erfc(2^58 / (sqrt 2 sigma))
  direct   : blind rotation of the LUT polynomial (identity LUT)
  multi    : multi-value outputs (w-step), per LUT norm^2
  sign     : sign-gate outputs
Usage: [FR_PARAMS=k2n1024] python3 tools/noise.py [count] [out.json]
"""
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import fheregex as F  # noqa: E402
import oracle_ffi as of  # noqa: E402

DELTA = 1 << 59


def signed(x):
    x = np.asarray(x, dtype=np.uint64)
    return x.view(np.int64).astype(np.float64)


def phase(lwe, s):
    s = np.asarray(s, dtype=np.uint64)
    a = lwe[..., :-1].astype(np.uint64)
    with np.errstate(over="ignore"):
        dot = (a * s).sum(axis=-1, dtype=np.uint64)
        return lwe[..., -1].astype(np.uint64) - dot


def stats(err):
    e = np.asarray(err, dtype=np.float64)
    return {"log2_std": math.log2(max(e.std(), 1.0)), "log2_max": math.log2(max(np.abs(e).max(), 1.0)), "count": int(e.size)}


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    key = of.load_fixture_key()
    s_big, s_small = key["s_big"], key["s_small"]
    with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
        blob = f.read()
    ring = {"fft": F.RING_FFT, "rns": F.RING_RNS}.get(os.environ.get("FR_RING", ""))
    k, N = (2, 1024) if os.environ.get("FR_PARAMS") == "k2n1024" else (1, 2048)
    ctx = F.Context(0, params=F.default_params(k=k, N=N, ring=ring))
    ctx.load_client_key(blob)
    ctx.gen_server_key(42)
    rng = np.random.default_rng(1)
    msgs = rng.integers(0, 16, count)
    fresh = ctx.encrypt_blocks([int(m) for m in msgs], seed=99)
    res = {}
    with np.errstate(over="ignore"):
        res["fresh"] = stats(signed(phase(fresh, s_big) - msgs.astype(np.uint64) * np.uint64(DELTA)))
        ks = ctx.dev_keyswitch(fresh)
        res["ks"] = stats(signed(phase(ks, s_small) - msgs.astype(np.uint64) * np.uint64(DELTA)))
        # modulus switch to 2N: round(x 2N / 2^64) per coefficient, phase in Z_2N
        l2 = int(math.log2(2 * N))
        ab = ((ks >> np.uint64(64 - l2 - 1)) + np.uint64(1)) >> np.uint64(1)
        ab &= np.uint64(2 * N - 1)
        ph = (ab[:, -1].astype(np.int64) - (ab[:, :-1].astype(np.int64) * s_small.astype(np.int64)).sum(axis=1)) % (2 * N)
        err = (ph - msgs.astype(np.int64) * (2 * N // 32)) % (2 * N)
        err = np.where(err >= N, err - 2 * N, err).astype(np.float64) * 2.0 ** (64 - l2)
        res["ms"] = stats(err)
        sd = float(np.std(err))
        res["ms"]["fail_per_bootstrap"] = math.erfc(2.0 ** 58 / (math.sqrt(2) * sd)) if sd > 0 else 0.0
        ident = [list(range(16))] * count
        out = ctx.dev_blind_rotate(ks, ident)
        res["direct"] = stats(signed(phase(out, s_big) - msgs.astype(np.uint64) * np.uint64(DELTA)))
        # multi-value: three LUTs of increasing ||w||^2 on each input
        luts = [[int(v == 5) for v in range(16)],          # ||w||^2 = 2
                [int(v >= 8) for v in range(16)],          # 2 (step + wrap)
                [v % 2 for v in range(16)]]                 # 16 (not merged by the executor; measured here)
        for li, lut in enumerate(luts):
            errs = []
            for i in range(min(count, 64)):
                o = ctx.dev_blind_rotate_multi(ks[i], [lut], direct=False)
                errs.append(signed(phase(o[0], s_big) - np.uint64(lut[msgs[i]] * DELTA)))
            norm2 = sum((lut[m] - lut[m - 1]) ** 2 for m in range(1, 16)) + (lut[0] + lut[15]) ** 2
            res[f"multi_norm2_{norm2}_{li}"] = stats(np.array(errs))
        errs = []
        for i in range(min(count, 64)):
            # sign gate on s = m - 7.5 (offset -15 in Delta/2 units): [m >= 8]
            lw = fresh[i].copy()
            lw[-1] = lw[-1] - np.uint64(15 << 58)
            k1 = ctx.dev_keyswitch(lw[None])
            o = ctx.dev_blind_rotate_multi(k1[0], [[0] * 16], direct=2)
            errs.append(signed(phase(o[0], s_big) - np.uint64(int(msgs[i] >= 8) * DELTA)))
        res["sign"] = stats(np.array(errs))
    res["threshold_log2"] = 58.0
    res["ring"] = "fft" if ctx.params.ring == F.RING_FFT else "rns"
    res["params"] = f"k{k}n{N}"
    print(json.dumps(res, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
