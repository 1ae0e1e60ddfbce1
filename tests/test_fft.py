"""FR_RING_FFT: the blind rotation on the 2^64 torus with an f64 negacyclic FFT
(tfhe-rs's own ring representation, reference Cargo.lock:602-615 / 110-114).

CPU: the oracle's FFT product against exact schoolbook products, the torus
server key identical between the product's keygen and the oracle's, the
oracle's blind rotation decrypting to the LUT values.  GPU: the device
blind rotation (direct, multi-value, sign) and gate programs bit-exact
against the oracle's restatement of the same operation sequence, and whole
matches decrypting to the reference result.  Both compiled points run: the
reference's k = 1, N = 2048 and BASELINE's "N = 1024" set (k = 2, N = 1024,
the same flattened 2048-bit key; ciphertext.rs:43-44 names the former)."""
import ctypes as C
import os

import numpy as np
import pytest

import fheregex as F
import oracle_ffi as of
import regex_oracle as ro
from conftest import GOLDEN

SEED = 42


POINTS = [(1, 2048), (2, 1024)]


@pytest.fixture(scope="module", params=POINTS, ids=["k1n2048", "k2n1024"])
def point(request):
    return request.param


@pytest.fixture(scope="module")
def oracle_fft(fixture_key, point):
    k, N = point
    return of.Oracle(fixture_key, seed=SEED, k=k, N=N, ring=of.RING_FFT)


def fft_mul(a, b):
    N = len(a)
    out = np.zeros(N, dtype=np.int64)
    p = lambda x: x.ctypes.data_as(C.POINTER(C.c_int64))
    a = np.ascontiguousarray(a, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.int64)
    of.lib().or_fft_ring_mul(N, p(a), p(b), p(out))
    return out


def schoolbook(a, b):
    N = len(a)
    out = [0] * N
    for i in range(N):
        ai = int(a[i])
        if ai == 0:
            continue
        for j in range(N):
            d = i + j
            if d < N:
                out[d] += ai * int(b[j])
            else:
                out[d - N] -= ai * int(b[j])
    return np.array([((x + (1 << 63)) % (1 << 64)) - (1 << 63) for x in out], dtype=np.int64)


@pytest.mark.parametrize("N,abits,bbits", [(16, 20, 10), (256, 22, 12), (2048, 22, 8)])
def test_fft_product_exact_for_small_operands(N, abits, bbits):
    """|a| |b| N < 2^50: the f64 FFT product rounds to the exact integer product."""
    rng = np.random.default_rng(N)
    a = rng.integers(-(1 << abits), 1 << abits, N, dtype=np.int64)
    b = rng.integers(-(1 << bbits), 1 << bbits, N, dtype=np.int64)
    if N == 2048:  # keep the schoolbook check fast: sparse a
        a[rng.random(N) < 0.9] = 0
    assert (fft_mul(a, b) == schoolbook(a, b)).all()


@pytest.mark.parametrize("N", [1024, 2048])
def test_fft_tables_closed_forms(N):
    """The kernel computes leaf exponents in closed form, L(j) = 1 + 4 brv(j) (the
    slot of X^e's factor psi^(e L)); the twiddles are psi^((M >> (s+1)) (4 brv_s(b) + 1))
    from the quadrant table, psi^(k + M q) = i^q psi^k exactly."""
    M = N // 2
    LOG = M.bit_length() - 1
    tw = np.zeros(2 * M)
    qt = np.zeros(N)
    leaf = np.zeros(M, dtype=np.uint16)
    of.lib().or_fft_tables(N, tw.ctypes.data_as(C.POINTER(C.c_double)), qt.ctypes.data_as(C.POINTER(C.c_double)),
                           leaf.ctypes.data_as(C.POINTER(C.c_uint16)))
    brv = lambda x, b: int(format(x, "0%db" % b)[::-1], 2) if b else 0
    assert all(int(leaf[j]) == 1 + 4 * brv(j, LOG) for j in range(M))
    twc, qtc = tw.view(np.complex128), qt.view(np.complex128)
    for s in range(LOG):
        for b in range(1 << s):
            q, r = divmod(((M >> (s + 1)) * (4 * brv(b, s) + 1)) % (2 * N), N // 2)
            z = qtc[r]
            for _ in range(q):
                z = complex(-z.imag, z.real)
            assert twc[(1 << s) + b] == z, (s, b)


def test_fft_monomial_is_a_rotation():
    N = 64
    rng = np.random.default_rng(3)
    a = rng.integers(-(1 << 20), 1 << 20, N, dtype=np.int64)
    for e in (0, 1, 17, 63):
        b = np.zeros(N, dtype=np.int64)
        b[e] = 1
        exp = np.concatenate([-a[N - e:], a[:N - e]]) if e else a
        assert (fft_mul(a, b) == exp).all(), e


def test_fft_error_on_torus_sized_products():
    """Digit-sized (2^22) times torus-sized (2^63) operands: the FFT result
    modulo 2^64 stays within 2^44 of the exact product (the noise budget the
    bootstrap relies on; tfhe-rs's FFT has the same error class)."""
    N = 2048
    rng = np.random.default_rng(5)
    a = rng.integers(-(1 << 22), 1 << 22, N, dtype=np.int64)
    a[rng.random(N) < 0.97] = 0
    b = rng.integers(-(1 << 62), 1 << 62, N, dtype=np.int64)
    err = (fft_mul(a, b) - schoolbook(a, b)).astype(np.int64)  # wraps mod 2^64
    assert np.abs(err).max() < (1 << 44), int(np.abs(err).max()).bit_length()


def test_torus_of_exact():
    L = of.lib()
    for v, e in [(0.0, 0), (-1.0, (1 << 64) - 1), (2.0**63, 1 << 63), (-(2.0**63), 1 << 63), (2.0**64 + 2**20, 1 << 20),
                 (3 * 2.0**70 + 5 * 2.0**30, (5 << 30) % (1 << 64)), (-(2.0**80) - 2.0**40, ((1 << 64) - (1 << 40)))]:
        assert L.or_torus_of(v) == e, (v, e)


def test_torus_server_key_matches_oracle(key_blob, oracle_fft, point):
    ctx = F.Context(device=-1, params=F.default_params(k=point[0], N=point[1], ring=F.RING_FFT))
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(SEED)
    ksk, bsk = ctx.export_server_key()
    assert (ksk == oracle_fft.ksk).all()
    assert (bsk == oracle_fft.bsk).all()


def test_torus_ggsw_rows_encrypt_gadget_times_key_bit(oracle_fft, fixture_key):
    """Row r of GGSW w decrypts (component phase) to m_w * 2^41 on component r's
    coefficient 0 plus small noise (k mask polynomials, body last)."""
    O = oracle_fft
    N, k = O.P.N, O.P.k
    kp1 = k + 1
    s = O.s_big.astype(np.int64).reshape(k, N)
    ss = O.s_small
    for w in (0, 1, 2, 99):
        t, g = divmod(w, 3)
        si, sj = int(ss[2 * t]), int(ss[2 * t + 1])
        m = [si & sj, si & (1 - sj), (1 - si) & sj][g]
        for r in range(kp1):
            row = O.bsk[(w * kp1 + r) * kp1 * N:(w * kp1 + r + 1) * kp1 * N].reshape(kp1, N)
            B = row[k].astype(np.uint64)
            # phase = B - sum_j A_j*S_j (negacyclic), mod 2^64, computed exactly with Python ints on a few coefficients
            for c in (0, 1, N - 1):
                acc = int(B[c])
                for j in range(k):
                    A = row[j].astype(np.uint64)
                    for u in np.nonzero(s[j])[0]:
                        src = c - u
                        acc -= int(A[src]) if src >= 0 else -int(A[src + N])
                acc %= 1 << 64
                # gadget on component r: +2^41 on the body (r = k) is +2^41 in the
                # phase; on mask j = r it is -2^41 * S_r[c] (X^0 times the key polynomial)
                expect = (m << 41) if (c == 0 and r == k) else (-(m << 41) * int(s[r][c]) if r < k else 0)
                err = (acc - expect) % (1 << 64)
                err = err - (1 << 64) if err >= 1 << 63 else err
                assert abs(err) < 1 << 20, (w, r, c)


@pytest.mark.parametrize("msgs", [[9, 3, 15, 0], [1, 2, 7, 12]])
def test_oracle_fft_blind_rotation_decrypts(oracle_fft, msgs):
    O = oracle_fft
    ks = O.keyswitch(O.encrypt_blocks(msgs, seed=sum(msgs)))
    lut = [(7 * m + 3) % 16 for m in range(16)]
    for i, m in enumerate(msgs):
        assert int(O.decode16(O.blind_rotate(ks[i], lut))[0]) == lut[m]
    luts = [lut, [m % 4 for m in range(16)], [int(m == msgs[0]) for m in range(16)]]
    got = O.blind_rotate_multi(ks[0], luts)
    assert [int(x) for x in O.decode16(got)] == [l[msgs[0]] for l in luts]


# ------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def fctx(key_blob, point):
    ctx = F.Context(device=0, params=F.default_params(k=point[0], N=point[1], ring=F.RING_FFT))
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(SEED)
    return ctx


@pytest.mark.gpu
def test_fft_device_info(fctx):
    assert "ring=fft" in fctx.info()


@pytest.mark.gpu
def test_fft_blind_rotate_bit_exact(fctx, oracle_fft):
    O = oracle_fft
    msgs = [5, 12, 0, 9]
    ks = O.keyswitch(O.encrypt_blocks(msgs, seed=31))
    luts = [[(3 * m + 1) % 16 for m in range(16)], [int(m >= 4) for m in range(16)], [m ^ 5 for m in range(16)],
            [15 - m for m in range(16)]]
    got = fctx.dev_blind_rotate(ks, luts)
    for i in range(len(msgs)):
        exp = O.blind_rotate(ks[i], luts[i])
        assert (got[i] == exp).all(), (i, int(np.count_nonzero(got[i] != exp)))
        assert O.decode16(got[i])[0] == luts[i][msgs[i]]


@pytest.mark.gpu
def test_fft_blind_rotate_random_masks_bit_exact(fctx, oracle_fft):
    """Uniformly random keyswitched LWEs (every mask coefficient nonzero with
    high probability, all 2N rotation amounts exercised)."""
    O = oracle_fft
    rng = np.random.default_rng(8)
    ks = rng.integers(0, 2**64 - 1, (3, O.n + 1), dtype=np.uint64, endpoint=True)
    ks[2, : O.n // 2] = 0  # half of the steps skipped
    luts = [[m for m in range(16)]] * 3
    got = fctx.dev_blind_rotate(ks, luts)
    for i in range(3):
        assert (got[i] == O.blind_rotate(ks[i], luts[i])).all(), i


@pytest.mark.gpu
def test_fft_multi_value_and_sign_bit_exact(fctx, oracle_fft):
    O = oracle_fft
    ks = O.keyswitch(O.encrypt_blocks([6, 13], seed=55))
    luts = [[int(v == 6) for v in range(16)], [int(v in (6, 13)) for v in range(16)], [int(v >= 9) for v in range(16)],
            [int(v == 13) for v in range(16)], [int(v % 2 == 0) for v in range(16)]]
    for i, m in enumerate([6, 13]):
        got = fctx.dev_blind_rotate_multi(ks[i], luts)
        exp = O.blind_rotate_multi(ks[i], luts)
        assert (got == exp).all(), i
        assert [int(O.decode16(o)[0]) for o in got] == [l[m] for l in luts]
        sg = fctx.dev_blind_rotate_multi(ks[i], [luts[0]], direct=2)
        assert (sg == O.blind_rotate_multi(ks[i], [luts[0]], direct=2)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("pattern,content", [("/abc/", "xyabcz"), ("/^abc$/", "abc"), ("/a[b-d]c/", "zzacczz"),
                                             ("/abc/", "xyabz!"), ("/the/i", "In ThE end")])
def test_fft_has_match_decrypts_to_reference(fctx, pattern, content):
    hs = fctx.upload_radix(fctx.encrypt_str(content, seed=4))
    out, st = fctx.has_match(hs, pattern)
    exp = ro.has_match(content, pattern)
    assert fctx.decrypt_radix(fctx.download_radix(out)) == exp.result
    assert (st.ct_ops, st.cache_hits) == (exp.ct_ops, exp.cache_hits)


@pytest.mark.gpu
def test_fft_metric_config_256_chars(fctx):
    rng = np.random.default_rng(0)
    s = list("".join(chr(c) for c in rng.integers(0x20, 0x7F, 256)))
    s[200:203] = "abc"
    s = "".join(s)
    hs = fctx.upload_radix(fctx.encrypt_str(s, seed=9))
    out, st = fctx.has_match(hs, "/abc/")
    assert fctx.decrypt_radix(fctx.download_radix(out)) == 1
    s2 = s.replace("abc", "abd")
    hs2 = fctx.upload_radix(fctx.encrypt_str(s2, seed=10))
    out2, _ = fctx.has_match(hs2, "/abc/")
    assert fctx.decrypt_radix(fctx.download_radix(out2)) == ro.has_match(s2, "/abc/").result



@pytest.mark.gpu
@pytest.mark.parametrize("keygen", [F.KEYGEN_AUTO, F.KEYGEN_HOST])
def test_fft_throughput_shape_bit_exact(key_blob, oracle_fft, point, keygen, monkeypatch):
    """The throughput shape on a batch large enough for it (300 > the latency shape's
    256; k = 1 with the pair shape off), with the Fourier key laid out by the device
    keygen and by the host upload: bit-exact against the oracle."""
    monkeypatch.setenv("FR_FFT_PAIR_BATCH", "0")
    ctx = F.Context(device=0, params=F.default_params(k=point[0], N=point[1], ring=F.RING_FFT))
    monkeypatch.delenv("FR_FFT_PAIR_BATCH")
    ctx.load_client_key(key_blob)
    ctx.set_keygen(keygen)
    ctx.gen_server_key(SEED)
    O = oracle_fft
    rng = np.random.default_rng(300)
    ks = rng.integers(0, 2**64 - 1, (300, O.n + 1), dtype=np.uint64, endpoint=True)
    luts = [[(5 * m + i) % 16 for m in range(16)] for i in range(300)]
    got = ctx.dev_blind_rotate(ks, luts)
    for i in (0, 1, 150, 299):
        assert (got[i] == O.blind_rotate(ks[i], luts[i])).all(), i


def _shape_ctx(key_blob, point, monkeypatch, **env):
    """A context whose launch-shape limits come from FR_FFT_* (read at creation)."""
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    ctx = F.Context(device=0, params=F.default_params(k=point[0], N=point[1], ring=F.RING_FFT))
    for k in env:
        monkeypatch.delenv(k)
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(SEED)
    return ctx


@pytest.mark.gpu
@pytest.mark.parametrize("point", [(1, 2048)], indirect=True, ids=["k1n2048"])  # a k = 1 geometry
@pytest.mark.parametrize("count", [301, 512])
def test_fft_pair_shape_bit_exact(key_blob, oracle_fft, point, monkeypatch, count):
    """The pair shape (k = 1: two bootstraps per workgroup sharing key loads, twiddles
    and barriers; an odd count's last workgroup holds one) bit-exact against the oracle
    on sampled rows and against the one-bootstrap throughput shape on every row, with
    zero pairs in one bootstrap's coefficients but not its partner's (steps the pair
    runs for one of them only)."""
    pair = _shape_ctx(key_blob, point, monkeypatch, FR_FFT_PAIR_BATCH=4096)
    tp = _shape_ctx(key_blob, point, monkeypatch, FR_FFT_PAIR_BATCH=0)
    O = oracle_fft
    rng = np.random.default_rng(count)
    ks = rng.integers(0, 2**64 - 1, (count, O.n + 1), dtype=np.uint64, endpoint=True)
    ks[0, 0:200] = 0  # bootstrap 0: 100 zero pairs its partner (1) does not have
    ks[3, 1:O.n] = 0  # bootstrap 3: a single nonzero coefficient
    luts = [[(3 * m + i) % 16 for m in range(16)] for i in range(count)]
    got = pair.dev_blind_rotate(ks, luts)
    assert (got == tp.dev_blind_rotate(ks, luts)).all()
    for i in (0, 1, 3, count // 2, count - 1):
        assert (got[i] == O.blind_rotate(ks[i], luts[i])).all(), i


@pytest.mark.gpu
@pytest.mark.parametrize("point", [(1, 2048)], indirect=True, ids=["k1n2048"])  # a k = 1 geometry
@pytest.mark.parametrize("count", [257, 512])
def test_fft_dual_shape_bit_exact(key_blob, oracle_fft, point, monkeypatch, count):
    """The dual shape (FR_FFT_DUAL=1, k = 1: one bootstrap per 4-wave workgroup, both
    polynomials in every lane, no MAC exchange, two workgroups per CU) bit-exact against
    the oracle on sampled rows and against the pair shape on every row, including rows
    with runs of zero pairs; and a whole /abc/ x 256 match bit-identical to the pair
    shape's."""
    dual = _shape_ctx(key_blob, point, monkeypatch, FR_FFT_DUAL=1)
    pair = _shape_ctx(key_blob, point, monkeypatch)
    O = oracle_fft
    rng = np.random.default_rng(count + 7)
    ks = rng.integers(0, 2**64 - 1, (count, O.n + 1), dtype=np.uint64, endpoint=True)
    ks[0, 0:200] = 0
    ks[3, 1:O.n] = 0
    luts = [[(7 * m + i) % 16 for m in range(16)] for i in range(count)]
    got = dual.dev_blind_rotate(ks, luts)
    assert (got == pair.dev_blind_rotate(ks, luts)).all()
    for i in (0, 1, 3, count // 2, count - 1):
        assert (got[i] == O.blind_rotate(ks[i], luts[i])).all(), i
    if count == 512:
        s = "".join(chr(c) for c in rng.integers(0x20, 0x7F, 256)).replace("abc", "abd")
        s = s[:150] + "abc" + s[153:]
        words = []
        for c in (dual, pair):
            o, _ = c.has_match(c.upload_radix(c.encrypt_str(s, seed=9)), "/abc/")
            words.append(c.download_radix(o))
        assert np.array_equal(words[0], words[1]) and dual.decrypt_radix(words[0]) == 1
