"""Product host logic through the C-ABI (no GPU): exports, parser, engine,
lowering, keygen and the host/device scalar maps, checked against the oracle."""
import ctypes
import json
import os
import random

import numpy as np
import pytest

import fheregex as F
import oracle_ffi as of
import regex_fuzz as rf
import regex_oracle as ro
from conftest import GOLDEN


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(F.LIB_PATH)
    syms = F.header_symbols()
    assert len(syms) >= 35
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) <= set(F._SIGS)


def test_host_only_context_fails_loudly_on_gpu_ops(key_blob):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    with pytest.raises(F.NoDevice):
        ctx.upload_radix(np.zeros((1, 4, ctx.lwe_len), dtype=np.uint64))
    with pytest.raises(F.NoDevice):
        ctx.dev_ring_mul(np.zeros(2048, np.uint64), np.zeros(2048, np.uint64))


def test_set_profiling_rejects_invalid_levels():
    """fr_set_profiling takes 0, 1 or 2; anything else is FR_ERR_INVALID,
    checked before the device, so a host-only context sees it too"""
    ctx = F.Context(device=-1)
    for bad in (-1, 3, 255):
        with pytest.raises(F.FheRegexError) as e:
            ctx.set_profiling(bad)
        assert not isinstance(e.value, F.NoDevice)
    with pytest.raises(F.NoDevice):
        ctx.set_profiling(1)


def test_set_lanes_validates():
    """fr_set_lanes takes 1..8 lanes and needs the device (host-only context: NoDevice)"""
    ctx = F.Context(device=-1)
    for bad in (0, -1, 9):
        with pytest.raises(F.FheRegexError) as e:
            ctx.set_lanes(bad)
        assert not isinstance(e.value, F.NoDevice)
    with pytest.raises(F.NoDevice):
        ctx.set_lanes(2)


@pytest.mark.parametrize("v", load("parser_vectors.json"), ids=lambda v: v["pattern"])
def test_parser_golden(v):
    assert F.parse(v["pattern"]) == v["ast"]


@pytest.mark.parametrize("mode", [F.LOWER_FAITHFUL, F.LOWER_THRESHOLD, F.LOWER_FAITHFUL_TREE])
@pytest.mark.parametrize("v", load("engine_vectors.json"), ids=lambda v: f'{v["content"]!r}-{v["pattern"]}')
def test_engine_golden(v, mode):
    r = F.plain_match(v["content"], v["pattern"], mode)
    assert (r.result_recorded, r.result_lowered, r.ct_ops, r.cache_hits) == (v["expected"], v["expected"], v["ct_ops"], v["cache_hits"])


@pytest.mark.parametrize("pattern,exc", [("/a{}/", F.ReferencePanic), ("/ab", F.ParseError), ("/[a-z0-9]/", F.ParseError),
                                         ("/^[a-z0-9]+$/", F.ParseError), ("/a+?/", F.ParseError), ("/a/x", F.ParseError),
                                         ("/a{99999999999999999999}/", F.ReferencePanic)])
def test_parse_errors_match_reference(pattern, exc):
    with pytest.raises(exc):
        F.parse(pattern)


def test_empty_seq_panics_like_reference():
    with pytest.raises(F.ReferencePanic):
        F.plain_match("a", "/^/")
    assert F.plain_match("", "/^/").result_recorded == 0


def test_fuzz_vs_oracle():
    rng = random.Random(7)
    n = 0
    while n < 400:
        p = rf.rand_pattern(rng)
        c = rf.rand_content(rng, rng.randint(0, 6))
        try:
            exp = ro.has_match(c, p)
            e_exc = None
        except (ro.ParseError, ro.ReferencePanic) as e:
            exp, e_exc = None, type(e).__name__
        if exp is not None and exp.n_branches > 500:
            continue
        for mode in (F.LOWER_FAITHFUL, F.LOWER_THRESHOLD, F.LOWER_FAITHFUL_TREE):
            try:
                r = F.plain_match(c, p, mode)
                got, g_exc = (r.result_recorded, r.result_lowered, r.ct_ops, r.cache_hits), None
            except (F.ParseError, F.ReferencePanic) as e:
                got, g_exc = None, type(e).__name__
            if e_exc or g_exc:
                assert e_exc == g_exc, (c, p)
            else:
                assert got == (exp.result, exp.result, exp.ct_ops, exp.cache_hits), (c, p, mode)
        n += 1


def test_config_counts_and_pbs():
    # reference ct_ops and the faithful build's PBS counts
    cases = [("abc", "/^abc$/", 5, 11), ("x" * 64, "/abc/", 371, 743), ("x" * 256, "/abc/", 1523, 3047),
             ("b" * 256, "/^[a-z]+$/", 1023, 2047), ("x" * 1024, "/the/i", 12263, 24527)]
    for c, p, ops, pbs in cases:
        r = F.plain_match(c, p, F.LOWER_FAITHFUL)
        assert (r.ct_ops, r.cache_hits, r.pbs) == (ops, 0, pbs), p
        t = F.plain_match(c, p, F.LOWER_THRESHOLD)
        assert t.ct_ops == ops and t.pbs < pbs and t.levels <= 6, (p, t.pbs, t.levels)


def test_faithful_tree_keeps_the_reference_op_mix():
    """FR_LOWER_FAITHFUL_TREE: the faithful gates (eq/gt/le = 3 PBS, and/or = 1), the same
    PBS count as FR_LOWER_FAITHFUL on every pattern, with the AND/OR chains of the
    reference's fold (engine.rs:22-35) rebalanced: log depth instead of #branches"""
    cases = [("abc", "/^abc$/", 11, 5), ("x" * 64, "/abc/", 743, 10), ("x" * 256, "/abc/", 3047, 12),
             ("b" * 256, "/^[a-z]+$/", 2047, 12), ("x" * 1024, "/the/i", 24527, 15)]
    for c, p, pbs, levels in cases:
        f = F.plain_match(c, p, F.LOWER_FAITHFUL)
        t = F.plain_match(c, p, F.LOWER_FAITHFUL_TREE)
        assert (t.ct_ops, t.pbs) == (f.ct_ops, f.pbs) == (t.ct_ops, pbs), p
        assert t.levels <= levels and t.levels <= f.levels, (p, t.levels, f.levels)
        assert t.result_lowered == f.result_lowered == f.result_recorded
    rng = random.Random(23)
    n = 0
    while n < 300:
        p = rf.rand_pattern(rng)
        c = rf.rand_content(rng, rng.randint(1, 10))
        try:
            f = F.plain_match(c, p, F.LOWER_FAITHFUL)
        except (F.ParseError, F.ReferencePanic):
            continue
        if f.n_branches > 500:
            continue
        t = F.plain_match(c, p, F.LOWER_FAITHFUL_TREE)
        assert (t.pbs, t.result_lowered) == (f.pbs, f.result_recorded), (c, p)
        assert t.levels <= f.levels, (c, p, t.levels, f.levels)
        n += 1


@pytest.mark.parametrize("content,pattern", [("q" * 100 + "abc" + "q" * 40, "/abc/"), ("b" * 90 + "z", "/^[a-z]+$/"),
                                             ("aaa" + "bcde" * 3 + "f", "/^a{2,8}(bc|de)+[^xyz]$/"),
                                             ("xx The end", "/the/i"), ("a" * 50 + "0", "/^[a-z]+$/")])
def test_large_plain_vs_oracle(content, pattern):
    exp = ro.has_match(content, pattern)
    r = F.plain_match(content, pattern)
    assert (r.result_recorded, r.result_lowered, r.ct_ops, r.cache_hits) == (exp.result, exp.result, exp.ct_ops, exp.cache_hits)


def test_start_range_partition_is_or():
    rng = random.Random(3)
    for _ in range(50):
        p = rf.rand_pattern(rng)
        c = rf.rand_content(rng, 9)
        try:
            full = F.plain_match(c, p).result_lowered
        except (F.ParseError, F.ReferencePanic):
            continue
        cut = rng.randint(0, len(c))
        a = F.plain_match(c, p, start_lo=0, start_hi=cut).result_lowered
        b = F.plain_match(c, p, start_lo=cut, start_hi=len(c)).result_lowered
        assert full == (a | b), (c, p, cut)


def test_match_parts_or_to_the_range_result():
    """fr_has_match_parts' program (host side): <= max_parts parts whose OR is the range's
    result (engine.rs:22-35 fold), on random patterns, ranges and part counts; faithful
    lowerings and max_parts = 1 give the one-output program unchanged"""
    rng = random.Random(31)
    n = 0
    while n < 300:
        p = rf.rand_pattern(rng)
        c = rf.rand_content(rng, rng.randint(1, 9))
        lo = rng.randint(0, len(c))
        hi = rng.randint(lo, len(c))
        P = rng.choice([1, 2, 3, 4, 8, 16])
        low = rng.choice([F.LOWER_THRESHOLD, F.LOWER_THRESHOLD, F.LOWER_FAITHFUL, F.LOWER_FAITHFUL_TREE])
        try:
            base = F.plain_match(c, p, low, start_lo=lo, start_hi=hi)
        except (F.ParseError, F.ReferencePanic):
            continue
        if base.n_branches > 500:
            continue
        r, vals = F.plain_match_parts(c, p, lo, hi, P, lowering=low)
        assert 1 <= len(vals) <= P and set(vals) <= {0, 1}, (c, p, P, vals)
        assert r.result_lowered == int(any(vals)) == base.result_lowered == base.result_recorded, (c, p, lo, hi, P)
        assert r.levels <= base.levels and r.pbs <= base.pbs, (c, p, P)
        if P == 1 or low != F.LOWER_THRESHOLD:
            assert len(vals) == 1 and (r.pbs, r.levels) == (base.pbs, base.levels), (c, p, P, low)
        n += 1


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_match_parts_save_the_combine_level(world):
    """/abc/ on 256 chars split by start offsets over `world` ranks with 16 // world parts
    each: every rank's program is one level shorter (the OR tree stops at its parts), so
    the ranks plus the one threshold OR over world * parts <= 16 booleans take the
    unsharded match's 4 levels, not 5; the parts' OR is the rank's range result"""
    import bench
    c = bench.make_content("printable", 256, seed=0)
    c = c[:77] + b"abc" + c[80:]
    P = 16 // world
    got = []
    for r in range(world):
        lo, hi = F.shard_starts(256, world, r)
        base = F.plain_match(c, "/abc/", start_lo=lo, start_hi=hi)
        pr, vals = F.plain_match_parts(c, "/abc/", lo, hi, P)
        assert (base.levels, pr.levels) == (4, 3) and len(vals) <= P, (r, base.levels, pr.levels, vals)
        assert pr.pbs == base.pbs - 1
        S = F.schedule_match(256, "/abc/", lo, hi, max_parts=P)
        assert len(S.parts) == len(vals) and len(S.level_off) - 1 == 3
        assert int(any(vals)) == base.result_recorded == int(any(c[i:i + 3] == b"abc" for i in range(lo, hi)))
        got.append(int(any(vals)))
    assert sum(got) >= 1 and F.plain_match(c, "/abc/").levels == 4


def test_enumeration_cost_counts_exactly():
    """FR_ENGINE_AUTO's decision: the reference enumeration's variant count (engine.rs:45-214,
    every spend of record_has_match) counted from the AST equals the count of actually
    enumerating, on random patterns, lengths, start ranges and caps (saturating alike past
    the cap); patterns whose enumeration panics give no count"""
    rng = random.Random(41)
    n = 0
    while n < 400:
        p = rf.rand_pattern(rng)
        L = rng.randint(0, 9)
        lo = rng.randint(0, L)
        hi = rng.randint(lo, L)
        cap = rng.choice([10, 100, 1000, 1 << 22])
        try:
            counted, enumerated = F.enumeration_cost(p, L, lo, hi, cap=cap, enumerate=True)
        except (F.ParseError, F.ReferencePanic):
            continue
        if counted is not None:
            assert counted == enumerated, (p, L, lo, hi, cap, counted, enumerated)
        n += 1
    for p, L, exp in [("/abc/", 256, 763), ("/the/i", 1024, 3067), ("/^a{2,8}(bc|de)+[^xyz]$/", 20, 12979)]:
        assert F.enumeration_cost(p, L, enumerate=True) == (exp, exp), p


def test_enumeration_cost_memory_bound(monkeypatch):
    """the counter's memo is bounded in bytes (entries and their stored end positions), and
    running out of it is its own outcome, distinct from "the enumeration would panic"; AUTO
    then enumerates under its own budget and so still takes the reference's decision"""
    pat, L = "/a*b*c*d*/", 300
    o, c, _ = F.enumeration_cost(pat, L, with_outcome=True)
    assert o == F.COST_COUNTED and c > 0
    o, c, _ = F.enumeration_cost(pat, L, mem_bytes=64 << 10, with_outcome=True)
    assert (o, c) == (F.COST_MEMORY, None)
    o, c, _ = F.enumeration_cost("/|a/", 4, with_outcome=True)  # empty Seq: engine.rs:189-190 panics
    assert (o, c) == (F.COST_PANIC, None)
    # AUTO with the counter starved: the same decision, counters and result as with it
    content = "xaabbcdyab"
    ref = F.plain_match(content, "/a*b*c*d*/", engine=F.ENGINE_AUTO)
    monkeypatch.setenv("FR_ENUM_COST_BYTES", str(64 << 10))
    got = F.plain_match(content, "/a*b*c*d*/", engine=F.ENGINE_AUTO)
    exp = ro.has_match(content, "/a*b*c*d*/")
    assert (got.ct_ops, got.cache_hits, got.result_recorded) == (ref.ct_ops, ref.cache_hits, ref.result_recorded) \
        == (exp.ct_ops, exp.cache_hits, exp.result)
    # past the enumeration budget (config 5 on 40 chars, ~2^22+ variants): merged, as with a count
    pat5 = "/^a{2,8}(bc|de)+[^xyz]$/"
    c5 = ("aaa" + "bcde" * 20)[:39] + "f"
    monkeypatch.setenv("FR_ENUM_COST_BYTES", "4096")
    assert F.enumeration_cost(pat5, 40, mem_bytes=4096) == (None, None)
    a = F.plain_match(c5, pat5, engine=F.ENGINE_AUTO)
    m = F.plain_match(c5, pat5, engine=F.ENGINE_MERGED)
    assert (a.result_recorded, a.ct_ops, a.pbs) == (m.result_recorded, m.ct_ops, m.pbs)
    assert a.result_recorded == ro.has_match_reach(c5, pat5) == 1


def test_auto_engine_skips_a_doomed_enumeration():
    """config 5 at its 512 chars: AUTO counts ~2^252 variants and goes straight to the
    merged evaluator (round 4 built 2^22 branches first: ~1 s of host time per cold call);
    the same result and circuit as FR_ENGINE_MERGED"""
    import time
    pat = "/^a{2,8}(bc|de)+[^xyz]$/"
    c = "aaa" + "bc" * 127 + "de" * 127 + "f"
    c = c[:512]
    assert F.enumeration_cost(pat, 512) == ((1 << 22) + 1, None)
    t = time.perf_counter()
    a = F.plain_match(c, pat, engine=F.ENGINE_AUTO)
    dt = time.perf_counter() - t
    m = F.plain_match(c, pat, engine=F.ENGINE_MERGED)
    assert (a.result_recorded, a.result_lowered, a.ct_ops, a.pbs, a.levels) == \
        (m.result_recorded, m.result_lowered, m.ct_ops, m.pbs, m.levels)
    assert dt < 0.5, dt
    # a pattern within the budget still enumerates (the reference's exact counters)
    e = F.plain_match("x" * 64 + "abc", "/abc/", engine=F.ENGINE_ENUMERATE)
    a = F.plain_match("x" * 64 + "abc", "/abc/", engine=F.ENGINE_AUTO)
    assert (a.ct_ops, a.cache_hits, a.n_branches) == (e.ct_ops, e.cache_hits, e.n_branches)


def test_match_parts_rejects_bad_counts():
    for P in (0, 17):
        with pytest.raises(F.FheRegexError):
            F.plain_match_parts("abcabc", "/abc/", 0, 6, P)
        with pytest.raises(F.FheRegexError):
            F.schedule_match(6, "/abc/", 0, 6, max_parts=P)


def test_scalar_maps_match_oracle():
    """Product scalar maps (Montgomery CRT, reciprocal digit, residue -> torus)
    vs the oracle's plain 128-bit definitions."""
    L, O = F.lib(), of.lib()
    Q = of.Q_RING
    g = O.or_pbs_gadget()
    rng = np.random.default_rng(9)
    xs = [0, 1, 2, Q - 1, Q - 2, Q // 2, Q // 2 + 1, g, g // 2, g // 2 + 1, Q - g // 2, Q - g // 2 - 1]
    xs += [int(v) for v in rng.integers(0, Q, 5000, dtype=np.uint64)]
    for x in xs:
        assert L.fr_debug_scalar(0, x, 0) == x  # CRT(x mod p0, x mod p1)
        assert L.fr_debug_scalar(1, x, 0) == O.or_decompose_pbs(x)
        assert L.fr_debug_scalar(2, x, 0) == O.or_conv(x)
    dig = (ctypes.c_int32 * 5)()
    for x in [int(v) for v in rng.integers(0, 2**64 - 1, 3000, dtype=np.uint64)] + [0, 2**64 - 1, 2**48, 2**63]:
        assert L.fr_debug_scalar(3, x, 12) == O.or_mod_switch(x, 12)
        O.or_ks_decompose(x, 3, 5, dig)
        for j in range(5):
            assert L.fr_debug_scalar(4, x, j) == (dig[j] & 0xFFFFFFFFFFFFFFFF)


def test_keygen_matches_oracle(key_blob, oracle_k1):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(42)
    ksk, bsk = ctx.export_server_key()
    assert ksk.shape == oracle_k1.ksk.shape and bsk.shape == oracle_k1.bsk.shape
    assert (ksk == oracle_k1.ksk).all()
    assert (bsk == oracle_k1.bsk).all()


def test_product_encrypt_matches_oracle(key_blob, oracle_k1):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    a = ctx.encrypt_str("abc~", seed=5)
    b = oracle_k1.encrypt_str(b"abc~", seed=5)
    assert (a == b).all()
    assert [ctx.decrypt_radix(a[i]) for i in range(4)] == list(b"abc~")
    with pytest.raises(ValueError):
        ctx.encrypt_str("caf\xe9", seed=1)


# --- state-merging engine -------------------------------

@pytest.mark.parametrize("mode", [F.LOWER_FAITHFUL, F.LOWER_THRESHOLD, F.LOWER_FAITHFUL_TREE])
@pytest.mark.parametrize("v", load("engine_vectors.json"), ids=lambda v: f'{v["content"]!r}-{v["pattern"]}')
def test_merged_engine_golden(v, mode):
    r = F.plain_match(v["content"], v["pattern"], mode, engine=F.ENGINE_MERGED)
    assert (r.result_recorded, r.result_lowered) == (v["expected"], v["expected"])


def test_merged_engine_fuzz_vs_oracle():
    """Merged engine vs the oracle's enumerator and its position-set simulator;
    start ranges random.  The merged engine refuses (FR_ERR_INVALID) only an
    unbounded repetition of a nullable operand holding an anchor, which the reference
    grammar cannot place inside a repetition: none of the 500 here (before round 3
    every unbounded repetition of a nullable operand was refused)."""
    rng = random.Random(19)
    n = refused = 0
    while n < 500:
        p = rf.rand_pattern(rng)
        c = rf.rand_content(rng, rng.randint(0, 8))
        lo = rng.randint(0, len(c))
        hi = rng.randint(lo, len(c))
        try:
            exp, e_exc = ro.has_match_reach(c, p, lo, hi), None
        except (ro.ParseError, ro.ReferencePanic) as e:
            exp, e_exc = None, type(e).__name__
        try:
            r = F.plain_match(c, p, F.LOWER_THRESHOLD, start_lo=lo, start_hi=hi, engine=F.ENGINE_MERGED)
            got, g_exc = (r.result_recorded, r.result_lowered), None
        except (F.ParseError, F.ReferencePanic) as e:
            got, g_exc = None, type(e).__name__
        except F.FheRegexError as e:
            assert e.code == -1 and "nullable" in str(e), (c, p)
            refused += 1
            n += 1
            continue
        if e_exc or g_exc:
            assert e_exc == g_exc, (c, p, lo, hi)
        else:
            assert got == (exp, exp), (c, p, lo, hi)
        n += 1
    assert refused == 0



def _config5(rng, L=512):
    body = "".join(rng.choice(["bc", "de"]) for _ in range((L - 4) // 2))
    return "aaa" + body + "f"


def test_config5_merged_engine():
    """BASELINE config 5 (/^a{2,8}(bc|de)+[^xyz]$/, 512 chars): the reference's
    enumeration exhausts memory; AUTO falls back to the merged engine, whose
    circuit is small and shallow, with the oracle simulator's result."""
    rng = random.Random(5)
    pat = "/^a{2,8}(bc|de)+[^xyz]$/"
    c = _config5(rng)
    assert len(c) == 512
    flips = [c[:-1] + "x", c[:200] + "q" + c[201:], "b" + c[1:], c[:3] + "cb" + c[5:]]
    for content in [c] + flips:
        exp = ro.has_match_reach(content, pat)
        r = F.plain_match(content, pat, engine=F.ENGINE_AUTO)
        assert (r.result_recorded, r.result_lowered) == (exp, exp), content[:12]
    assert ro.has_match_reach(c, pat) == 1 and ro.has_match_reach(flips[0], pat) == 0
    r = F.plain_match(c, pat, engine=F.ENGINE_MERGED)
    assert r.pbs < 20000 and r.levels <= 40, (r.pbs, r.levels)


def test_auto_engine_keeps_reference_counts_when_enumerable():
    a = F.plain_match("x" * 64, "/abc/", engine=F.ENGINE_AUTO)
    assert (a.ct_ops, a.cache_hits) == (371, 0)


def test_merged_nullable_unbounded_repetition_vs_oracle():
    """Unbounded repetitions of nullable operands in the merged engine (round 3): the
    reference's per-entry count range [max(1, lo), L - p] (engine.rs:127-183) empties
    near the end of the content when lo > L - p; every start range of every content
    of up to 7 chars over a small alphabet, against the position-set simulator."""
    import itertools
    pats = ["/(a?){3,}$/", "/(b?c?){2,}/", "/x(a?)+$/", "/(.{,})+/", "/((ab)?){4,}c/", "/^(a(.{,})+|[^f-h]*[ac]+)/",
            "/(a*b?)+x/i", "/(c?){5,}/"]
    rng = random.Random(5)
    for pat in pats:
        for n in range(8):
            for c in rng.sample(list(itertools.product("abcx", repeat=n)), min(6, 4 ** n)):
                c = "".join(c)
                for lo in sorted({0, n // 2, max(0, n - 2), n}):
                    exp = ro.has_match_reach(c, pat, lo, n)
                    r = F.plain_match(c, pat, F.LOWER_THRESHOLD, start_lo=lo, start_hi=n, engine=F.ENGINE_MERGED)
                    assert (r.result_recorded, r.result_lowered) == (exp, exp), (pat, c, lo)


def test_fuzz_scale_lowering_vs_oracle():
    """The product's engine + lowering (plaintext semantics, fr_plain_match) on the
    fuzz-at-scale fixture (64-300 chars; tests/golden/make_fuzz_scale.py) against
    the oracle's position-set simulator results."""
    with open(os.path.join(GOLDEN, "fuzz_scale.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == 20
    for c in cases:
        pm = F.plain_match(c["content"].encode(), c["pattern"], engine=F.ENGINE_AUTO)
        assert pm.result_lowered == pm.result_recorded == c["expected"], c["pattern"]


def test_fuzz_boundary_lowering_vs_oracle():
    """The same on the boundary fixture (256-512 chars, a witness or a near miss of it
    planted at the first or last start offsets; tests/golden/make_fuzz_boundary.py):
    every third case here (the CPU suite's time budget), all 30 on the GPU."""
    with open(os.path.join(GOLDEN, "fuzz_boundary.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == 30
    for c in cases[::3]:
        pm = F.plain_match(c["content"].encode(), c["pattern"], engine=F.ENGINE_AUTO)
        assert pm.result_lowered == pm.result_recorded == c["expected"], (c["pattern"], c["at"])


def test_c_abi_consumer(tmp_path):
    """include/fheregex.h from plain C99 (gcc -Werror) against the in-tree library: a
    host-only context, the reference's parse Err, golden counters, the fixture key,
    FR_ERR_NO_DEVICE on GPU entry points (tests/c_abi_consumer.c)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    lib_dir = os.path.join(repo, "fhe-regex_amd")
    exe = str(tmp_path / "c_abi_consumer")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(repo, "include"),
                    os.path.join(here, "c_abi_consumer.c"), "-o", exe, "-L", lib_dir, "-lfheregex",
                    "-Wl,-rpath," + lib_dir, "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    res = subprocess.run([exe, os.path.join(GOLDEN, "client_key")], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    assert "ok" in res.stdout
