"""The f64 blind rotation pinned to exact arithmetic (VERDICT r05 "weak" 1).

Every other blind-rotation test compares the device with the oracle's f64 ladder
(oracle/tfhe_oracle.c blind_rotate_torus), which restates the product's own f64
operation sequence (csrc/fft.h), so "bit-exact" there shows the device implements
the spec.  Here the spec itself is checked against an independent ladder,
or_blind_rotate_exact: the same unrolled CMUX steps with an u64 accumulator and
schoolbook negacyclic products mod 2^64 -- no floating point anywhere.

Two properties, because the two ladders cannot agree word for word over many steps:
a gadget digit is the top 23 bits of an accumulator coefficient, and where the f64
value sits within its rounding error of a digit boundary the two ladders take
neighbouring digits; the step's output then differs by one GGSW row (a fresh
encryption: uniform mask words), and from there on the two accumulators are
different, equally valid encryptions.

1. One step, word for word.  A keyswitched LWE with a single non-zero pair of
   mask coefficients runs exactly one step (zero pairs are skipped, as in the
   oracle and the kernels), from the exact LUT polynomial.  Sample extraction of a
   direct LUT exposes every mask coefficient of the GLWE accumulator (and the
   body's coefficient 0), so each of the k*N + 1 output words is compared:
   |f64 - exact| <= 2^44, the per-product bound of DESIGN §2.1 (the f64 FFT
   product of a digit polynomial, |d| <= 2^22, with a torus polynomial; a step's
   MAC accumulates its products in the Fourier domain before one inverse
   transform).  Measured: 2^41.6 (k = 1), 2^40.7 (k = 2).
2. A whole ladder, in distribution.  Over fresh encryptions the output phase error
   (phase - LUT value * Delta) of the f64 ladder and of the exact ladder: every
   output decodes to its LUT value under both, and the f64 ladder's error standard
   deviation stays within sqrt(sigma_exact^2 + steps * (|s| + 1) * eps^2): the
   f64 ladder's own error, independent per step and coefficient, seen through the
   phase b - <a, s>, with eps = 2^41 per coefficient and step.  (Measured one step
   from the LUT polynomial, whose mask is zero: 2^39.1 rms, 2^41.6 max; from a
   full-magnitude accumulator the products are ~2^1.2 larger, and the whole-ladder
   excess below puts the steady-state rms near 2^40.3.)  The bound is about 1.8
   bits above the exact ladder's std; measured: 2^49.5 against 2^48.6 (k = 1),
   2^49.0 against 2^48.6 (k = 2).  And the largest error stays 5 bits below the
   decoding threshold Delta/2 = 2^58.

Reference: tfhe-rs 0.2 computes the same external products with its own f64 FFT
(concrete-fft 0.1.0, reference Cargo.lock:110-114); the reference's tests pin only
decrypted bits (src/regex/engine.rs:281-290), which is what this closes the gap to.
"""
import math

import numpy as np
import pytest

import fheregex as F
import oracle_ffi as of

SEED = 42
POINTS = [(1, 2048), (2, 1024)]
ONE_STEP_BOUND = 2.0 ** 44


@pytest.fixture(scope="module", params=POINTS, ids=["k1n2048", "k2n1024"])
def point(request):
    return request.param


@pytest.fixture(scope="module")
def oracle_fft(fixture_key, point):
    k, N = point
    return of.Oracle(fixture_key, seed=SEED, k=k, N=N, ring=of.RING_FFT)


def one_step_inputs(O, count, seed):
    """keyswitched LWEs with one non-zero mask pair each (one blind-rotation step),
    random body; random direct LUTs"""
    rng = np.random.default_rng(seed)
    ks = np.zeros((count, O.n + 1), dtype=np.uint64)
    for q in range(count):
        i = 2 * int(rng.integers(0, O.n // 2))
        ks[q, i:i + 2] = rng.integers(0, 2**64 - 1, 2, dtype=np.uint64, endpoint=True)
        ks[q, -1] = rng.integers(0, 2**64 - 1, dtype=np.uint64, endpoint=True)
    luts = rng.integers(0, 16, (count, 16), dtype=np.uint8)
    return ks, luts


def word_gap(a, b):
    return int(np.abs((np.asarray(a, np.uint64) - np.asarray(b, np.uint64)).view(np.int64)).max())


def phase_errors(O, lwes, expected):
    exp = np.asarray(expected, dtype=np.uint64) << np.uint64(59)
    return (O.phase(lwes) - exp).view(np.int64).astype(np.float64)


def noise_bound_std(O, std_exact):
    """sqrt(std_exact^2 + steps * (|s| + 1) * eps^2): the f64 ladder's independent
    per-step error (eps = 2^41 rms per coefficient) seen through the phase
    b - <a, s> of every step's update"""
    steps = (O.n + 1) // 2
    weight = int(np.asarray(O.s_big).sum())
    eps = 2.0 ** 41
    return math.sqrt(std_exact ** 2 + steps * (weight + 1) * eps ** 2)


def test_exact_ladder_one_step_words(oracle_fft):
    """the f64 ladder (the device's spec) against the exact ladder, one step, every word"""
    O = oracle_fft
    ks, luts = one_step_inputs(O, 12, seed=1)
    ex = O.blind_rotate_exact(ks, luts, direct=1)[:, 0]
    worst = 0
    for q in range(len(ks)):
        f = O.blind_rotate(ks[q], list(luts[q]))
        worst = max(worst, word_gap(f, ex[q]))
        assert int(O.decode16(ex[q])[0]) == int(O.decode16(f)[0])
    assert worst <= ONE_STEP_BOUND, math.log2(worst)


def test_exact_ladder_no_step_is_exact(oracle_fft):
    """with every mask pair zero no step runs: the f64 and exact ladders return the rotated
    LUT polynomial, word for word (the f64 accumulator holds it exactly)"""
    O = oracle_fft
    rng = np.random.default_rng(2)
    ks = np.zeros((3, O.n + 1), dtype=np.uint64)
    ks[:, -1] = rng.integers(0, 2**64 - 1, 3, dtype=np.uint64, endpoint=True)
    luts = rng.integers(0, 16, (3, 16), dtype=np.uint8)
    ex = O.blind_rotate_exact(ks, luts, direct=1)[:, 0]
    for q in range(3):
        assert word_gap(O.blind_rotate(ks[q], list(luts[q])), ex[q]) == 0


def test_exact_ladder_multi_value_and_sign(oracle_fft):
    """the w-step (multi-value outputs) and the sign gate after an exact ladder decode like
    the f64 ladder's"""
    O = oracle_fft
    rng = np.random.default_rng(3)
    msgs = rng.integers(0, 16, 2)
    ks = O.keyswitch(O.encrypt_blocks(msgs, seed=4))
    luts = [[(m * 3 + f) % 2 for m in range(16)] for f in range(3)]
    ex = O.blind_rotate_exact(ks, np.array([luts, luts], dtype=np.uint8), direct=0)
    for q in range(2):
        f64 = O.blind_rotate_multi(ks[q], luts)
        assert list(O.decode16(ex[q])) == list(O.decode16(f64)) == [luts[f][msgs[q]] for f in range(3)]
    sg = O.blind_rotate_exact(ks, np.zeros((2, 1, 16), np.uint8), direct=2)[:, 0]
    for q in range(2):
        assert int(O.decode16(sg[q])[0]) == int(O.decode16(O.blind_rotate_multi(ks[q], [[0] * 16], direct=2))[0])


@pytest.mark.slow
def test_exact_ladder_noise_distribution(oracle_fft):
    """whole ladders on fresh encryptions: both decode, the f64 error std within the bound,
    the largest error 5 bits below Delta/2 (CPU: the oracle's f64 ladder, bit-identical to
    the device's)"""
    O = oracle_fft
    count = 12
    rng = np.random.default_rng(5)
    msgs = rng.integers(0, 16, count)
    ks = O.keyswitch(O.encrypt_blocks(msgs, seed=6))
    luts = rng.integers(0, 16, (count, 16), dtype=np.uint8)
    exp = [int(luts[q][msgs[q]]) for q in range(count)]
    ex = O.blind_rotate_exact(ks, luts, direct=1)[:, 0]
    f64 = np.stack([O.blind_rotate(ks[q], list(luts[q])) for q in range(count)])
    assert list(O.decode16(ex)) == exp == list(O.decode16(f64))
    ee, ef = phase_errors(O, ex, exp), phase_errors(O, f64, exp)
    assert ef.std() <= noise_bound_std(O, ee.std()), (math.log2(ef.std()), math.log2(ee.std()))
    assert np.abs(ef).max() < 2.0 ** 53


# ------------------------------------------------------------------ the device
def _ctx(key_blob, point, monkeypatch, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    ctx = F.Context(device=0, params=F.default_params(k=point[0], N=point[1], ring=F.RING_FFT))
    for k in env:
        monkeypatch.delenv(k)
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(SEED)
    return ctx


# (launch shape, count, env): the latency shape (<= 256 bootstraps, one per CU), the pair
# shape (k = 1 above 256: two per workgroup), the throughput shape (FR_FFT_PAIR_BATCH=0:
# two workgroups per CU) and the dual shape (FR_FFT_DUAL=1, k = 1)
SHAPES = [("latency", 24, {}), ("pair", 300, {}), ("throughput", 300, {"FR_FFT_PAIR_BATCH": 0}),
          ("dual", 300, {"FR_FFT_DUAL": 1})]


SHAPE_CASES = [((1, 2048), s) for s in SHAPES] + [((2, 1024), s) for s in SHAPES if s[0] in ("latency", "throughput")]


@pytest.mark.gpu
@pytest.mark.parametrize("point,shape", SHAPE_CASES, indirect=["point"],
                         ids=[f"k{p[0]}n{p[1]}-{s[0]}" for p, s in SHAPE_CASES])
def test_device_one_step_against_exact(key_blob, oracle_fft, point, monkeypatch, shape):
    """every launch shape (pair and dual: k = 1 geometries), one-step ladders: each output
    word of the device within 2^44 of the exact ladder's"""
    name, count, env = shape
    ctx = _ctx(key_blob, point, monkeypatch, **env)
    O = oracle_fft
    ks, luts = one_step_inputs(O, count, seed=10 + count)
    dev = ctx.dev_blind_rotate(ks, luts)
    ex = O.blind_rotate_exact(ks, luts, direct=1)[:, 0]
    gaps = [word_gap(dev[q], ex[q]) for q in range(count)]
    assert max(gaps) <= ONE_STEP_BOUND, (name, math.log2(max(gaps)))
    print(f"{name} k={point[0]}: max |device - exact| = 2^{math.log2(max(gaps) or 1):.2f} over {count} one-step ladders")


@pytest.mark.gpu
def test_device_full_ladder_noise_against_exact(key_blob, oracle_fft, point, monkeypatch):
    """whole ladders on the device (latency shape) against exact ladders on the same inputs:
    both decode to the LUT values, the device's error std within noise_bound_std of the
    exact ladder's, the largest error 5 bits below Delta/2"""
    ctx = _ctx(key_blob, point, monkeypatch)
    O = oracle_fft
    count = 32
    rng = np.random.default_rng(20)
    msgs = rng.integers(0, 16, count)
    ks = O.keyswitch(O.encrypt_blocks(msgs, seed=21))
    luts = rng.integers(0, 16, (count, 16), dtype=np.uint8)
    exp = [int(luts[q][msgs[q]]) for q in range(count)]
    dev = ctx.dev_blind_rotate(ks, luts)
    ex = O.blind_rotate_exact(ks, luts, direct=1)[:, 0]
    assert list(O.decode16(dev)) == exp == list(O.decode16(ex))
    ed, ee = phase_errors(O, dev, exp), phase_errors(O, ex, exp)
    bound = noise_bound_std(O, ee.std())
    print(f"k={point[0]}: error std device 2^{math.log2(ed.std()):.2f}, exact 2^{math.log2(ee.std()):.2f}, "
          f"bound 2^{math.log2(bound):.2f}; max device 2^{math.log2(np.abs(ed).max()):.2f}")
    assert ed.std() <= bound
    assert np.abs(ed).max() < 2.0 ** 53
