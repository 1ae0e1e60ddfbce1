"""The oracle itself, pinned against the reference's own vectors and fixture."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as of
import regex_oracle as ro
from conftest import GOLDEN


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("v", load("parser_vectors.json"), ids=lambda v: v["pattern"])
def test_oracle_parser_golden(v):
    # src/regex/parser.rs:358-678
    assert str(ro.parse(v["pattern"])) == v["ast"]


@pytest.mark.parametrize("v", load("engine_vectors.json"), ids=lambda v: f'{v["content"]!r}-{v["pattern"]}')
def test_oracle_engine_golden(v):
    # src/regex/engine.rs:256-280 results; SURVEY App. B counts
    r = ro.has_match(v["content"], v["pattern"])
    assert (r.result, r.ct_ops, r.cache_hits) == (v["expected"], v["ct_ops"], v["cache_hits"])


@pytest.mark.parametrize("pattern,err", [("/a{}/", ro.ReferencePanic), ("/ab", ro.ParseError), ("/[a-z0-9]/", ro.ParseError),
                                         ("/^[a-z0-9]+$/", ro.ParseError), ("/a+?/", ro.ParseError), ("/1/", ro.ParseError),
                                         ("/a/x", ro.ParseError), ("/[]/", ro.ParseError), ("/(a/", ro.ParseError)])
def test_oracle_parse_errors(pattern, err):
    with pytest.raises(err):
        ro.parse(pattern)


def test_oracle_empty_seq_panics():
    assert str(ro.parse("/^/")) == "Seq(SOF,Seq())"
    with pytest.raises(ro.ReferencePanic):
        ro.has_match("a", "/^/")
    assert ro.has_match("", "/^/").result == 0  # p >= L short-circuits before the panic


def test_config_counts():
    # SURVEY §8(a) op-count table (reference-faithful)
    assert (lambda r: (r.ct_ops, r.cache_hits))(ro.has_match("abc", "/^abc$/")) == (5, 0)
    assert ro.has_match("x" * 64, "/abc/").ct_ops == 371
    assert ro.has_match("x" * 256, "/abc/").ct_ops == 1523
    assert ro.has_match("b" * 256, "/^[a-z]+$/").ct_ops == 1023


def test_fixture_key_layout(fixture_key):
    k = fixture_key
    assert (k["n"], k["k"], k["N"]) == (742, 1, 2048)
    assert (k["pbs_base_log"], k["pbs_level"], k["ks_base_log"], k["ks_level"]) == (23, 1, 3, 5)
    assert (k["message_modulus"], k["carry_modulus"], k["num_blocks"]) == (4, 4, 4)
    assert int(k["s_big"].sum()) == 1031 and int(k["s_small"].sum()) == 395
    assert (k["glwe"] == k["s_big"]).all()


def test_ring_mul_vs_schoolbook():
    L = of.lib()
    rng = np.random.default_rng(3)
    for N in (16, 256):
        a = rng.integers(0, of.Q_RING, N, dtype=np.uint64)
        b = rng.integers(0, of.Q_RING, N, dtype=np.uint64)
        o1 = np.zeros(N, np.uint64)
        o2 = np.zeros(N, np.uint64)
        L.or_ring_mul(N, of.ptr(a), of.ptr(b), of.ptr(o1))
        L.or_ring_mul_schoolbook(N, of.ptr(a), of.ptr(b), of.ptr(o2))
        assert (o1 == o2).all()
    # pure-python negacyclic product for a tiny case
    N, P = 8, of.Q_RING
    a = rng.integers(0, P, N, dtype=np.uint64)
    b = rng.integers(0, P, N, dtype=np.uint64)
    ref = [0] * N
    for i in range(N):
        for j in range(N):
            m = int(a[i]) * int(b[j]) % P
            if i + j < N:
                ref[i + j] = (ref[i + j] + m) % P
            else:
                ref[i + j - N] = (ref[i + j - N] - m) % P
    o = np.zeros(N, np.uint64)
    L.or_ring_mul_schoolbook(N, of.ptr(a), of.ptr(b), of.ptr(o))
    assert [int(x) for x in o] == ref


def test_decompose_and_conv_properties():
    """Gadget digit and Z_Q -> torus map, against their exact definitions."""
    L = of.lib()
    Q = of.Q_RING
    p0, p1 = of.RNS_PRIMES
    assert L.or_q_modulus() == Q
    g = L.or_pbs_gadget()
    assert g == round(Q / 2**23) == (Q + 2**22) >> 23
    rng = np.random.default_rng(5)
    xs = [0, 1, g // 2, g // 2 + 1, g - 1, Q - 1, Q - 2, Q - g // 2, Q - g // 2 - 1, Q // 2, Q // 2 + 1]
    xs += [int(x) for x in rng.integers(0, Q, 2000, dtype=np.uint64)]
    p1m = (2**61 + p1 // 2) // p1
    for x in xs:
        d = L.or_decompose_pbs(x)
        ds = d if d < 2**63 else d - 2**64
        k = (x - x % p0) // p0
        t = (k * p1m + 2**37) >> 38
        assert ds == (t - 2**23 if t >= 2**22 else t)
        assert -(2**22) <= ds < 2**22
        err = (x - ds * g) % Q  # approximate-gadget error, centred mod Q
        err = err if err <= Q // 2 else err - Q
        assert abs(err) <= 0.51 * g
        y = L.or_conv(x)
        u0 = x % p0 * pow(p1, -1, p0) % p0
        u1 = x % p1 * pow(p0, -1, p1) % p1
        exp = (((u0 << 64) + (p0 - 1) // 2) // p0 + ((u1 << 64) + (p1 - 1) // 2) // p1) % 2**64
        assert y == exp
        # within one unit of round(x * 2^64 / Q) on the torus
        r = ((x << 64) + Q // 2) // Q % 2**64
        assert min((y - r) % 2**64, (r - y) % 2**64) <= 1


def test_encrypt_decrypt_roundtrip(oracle_k1):
    ct = oracle_k1.encrypt_str(b"Hello, World~", seed=11)
    assert bytes(oracle_k1.decrypt_radix(ct[i]) for i in range(ct.shape[0])) == b"Hello, World~"
    t = oracle_k1.trivial_blocks([1, 2, 3, 0])
    assert oracle_k1.decrypt_radix(t) == 1 + 2 * 4 + 3 * 16


@pytest.fixture(params=["fft", "rns"])
def oracle_ring(request, oracle_k1, oracle_rns):
    return oracle_k1 if request.param == "fft" else oracle_rns


def test_oracle_pbs_lut(oracle_ring):
    """KS -> BR -> SE on fresh and trivial inputs decrypts to the LUT value."""
    O = oracle_ring
    msgs = [0, 5, 15, 9]
    blocks = O.encrypt_blocks(msgs, seed=21)
    blocks[3] = O.trivial_blocks([9])[0]
    luts = [[(3 * m + 1) % 16 for m in range(16)], [m ^ 1 for m in range(16)], list(range(16)), [1] * 16]
    gates = [([(i, 1)], 0, luts[i]) for i in range(4)]  # offsets in units of Delta/2
    out = O.gates(gates, blocks)
    dec = O.decode16(out)
    assert [int(d) for d in dec] == [luts[i][msgs[i]] for i in range(4)]
    # trivial input: bootstrapping a trivial ciphertext yields a trivial (noiseless) one
    assert (out[3][:-1] == 0).all()


def test_oracle_multi_value_bootstrap(oracle_ring):
    """One rotation of (Delta/2)*u serves several LUTs (w_f factorization)."""
    O = oracle_ring
    ks = O.keyswitch(O.encrypt_blocks([7, 0], seed=41))
    luts = [[int(v == 7) for v in range(16)], [int(v in (5, 7)) for v in range(16)], [int(v >= 3) for v in range(16)],
            [int(v == 0) for v in range(16)]]
    for i, m in enumerate([7, 0]):
        outs = O.blind_rotate_multi(ks[i], luts)
        assert [int(O.decode16(o)[0]) for o in outs] == [l[m] for l in luts]
    # the factorization itself: (Delta/2) u * w_f == V_f in Z[X]/(X^N+1) (N small, exact)
    N, box, half = 64, 4, 2
    for lut in luts + [[(3 * v + 1) % 16 for v in range(16)]]:
        V = [2 * (lut[(j + half) // box] if (j + half) // box < 16 else -lut[0]) for j in range(N)]
        w = [0] * N
        for pos, d in of.lut_terms(N, lut):
            w[pos] += d
        prod = [0] * N
        for j in range(N):
            for i, d in enumerate(w):
                if d:
                    k = i + j
                    if k < N:
                        prod[k] += d
                    else:
                        prod[k - N] -= d
        assert prod == V


def test_oracle_sign_gate_fanin16(oracle_ring):
    """Sign gates: OR/AND of 16 booleans in one bootstrap (offset in Delta/2 units)."""
    O = oracle_ring
    bits = [0] * 16
    ct = O.encrypt_blocks(bits, seed=61)
    ct1 = ct.copy()
    ct1[9] = O.encrypt_blocks([1], seed=62)[0]
    ones = O.encrypt_blocks([1] * 16, seed=63)
    ins = [(i, 1) for i in range(16)]
    jobs = [(ins, -1, [0] * 16, 2), (ins, 1 - 32, [0] * 16, 2)]  # OR: s - 1/2 ; AND: s - 16 + 1/2
    out0 = O.gates(jobs, ct)
    out1 = O.gates(jobs, ct1)
    out2 = O.gates(jobs, ones)
    dec = lambda o: [int(O.decode16(x)[0]) for x in o]
    assert dec(out0) == [0, 0] and dec(out1) == [1, 0] and dec(out2) == [1, 1]


@pytest.mark.parametrize("v", load("engine_vectors.json"), ids=lambda v: f'{v["content"]!r}-{v["pattern"]}')
def test_reach_simulator_golden(v):
    # the position-set simulator (checker of the merged engine) on the reference's vectors
    assert ro.has_match_reach(v["content"], v["pattern"]) == v["expected"]


def test_reach_simulator_vs_enumerator_fuzz():
    """Pins has_match_reach to the reference-faithful enumerator (has_match):
    same result and same panics on fuzzed patterns/contents."""
    import random

    import regex_fuzz as rf
    rng = random.Random(11)
    n = 0
    while n < 300:
        p = rf.rand_pattern(rng)
        c = rf.rand_content(rng, rng.randint(0, 7))
        try:
            exp, e_exc = ro.has_match(c, p).result, None
        except (ro.ParseError, ro.ReferencePanic) as e:
            exp, e_exc = None, type(e).__name__
        try:
            got, g_exc = ro.has_match_reach(c, p), None
        except (ro.ParseError, ro.ReferencePanic) as e:
            got, g_exc = None, type(e).__name__
        assert (got, g_exc) == (exp, e_exc), (c, p)
        n += 1


def test_readme_semantics_vectors():
    """The reference README's documented semantics (README.md:33-58, transcribed by
    tests/golden/make_readme_vectors.py): the oracle and the product's recorded and lowered
    circuits (both engines) give the README's claim on every case, except the two where the
    code itself differs (ct_ge calls smart_gt, execution.rs:93), which follow the code."""
    import json
    import fheregex as F
    with open(os.path.join(GOLDEN, "readme_vectors.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == 100
    quirks = 0
    for c in cases:
        exp = c.get("code", c["readme"])
        quirks += "code" in c
        assert ro.has_match(c["content"], c["pattern"]).result == exp, c
        for eng in (F.ENGINE_ENUMERATE, F.ENGINE_MERGED):
            r = F.plain_match(c["content"], c["pattern"], engine=eng)
            assert (r.result_recorded, r.result_lowered) == (exp, exp), (c, eng)
    assert quirks == 2
