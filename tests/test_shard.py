"""One match split across ranks (fheregex.h fr_shard_* / fr_schedule_match).

The reference ORs one branch set per start offset (engine.rs:15-35); anchored
patterns have a single start (engine.rs:51-57), so start-offset sharding leaves
their work on one rank.  Level sharding splits every dependency level of the
lowered circuit into contiguous job slices and all-gathers each level's output
LWEs.  Here:
  * CPU: the schedule's plaintext semantics equal the lowered program's
    (fr_plain_match) and the job slices partition every level;
  * CPU, world-size-2 gloo: real LWE ciphertexts, each rank evaluating its
    slices with the CPU oracle (test infrastructure) and all-gathering the
    outputs; the result decrypts to the plaintext oracle's bit and is
    bit-identical to the unsharded evaluation of the same schedule;
  * GPU: the fr_shard_* path with two contexts on device 0 standing in for two
    ranks (device-to-device export/import), bit-identical to fr_has_match.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "fhe-regex_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import fheregex as F  # noqa: E402
import regex_oracle as ro  # noqa: E402

SEED = 42
CONFIG3 = "/^[a-z]+$/"
CONFIG5 = "/^a{2,8}(bc|de)+[^xyz]$/"
GLOO_CASES = [("bcdefg", CONFIG3), ("bcDefg", CONFIG3), ("aabcdef", CONFIG5), ("aabcdex", CONFIG5)]


def plain_schedule(S: F.Schedule, content: bytes) -> int:
    """Plaintext evaluation of a schedule (fr_job semantics, fheregex.h)."""
    val = {}

    def ref(r):
        if r >= 0:
            return val[r]
        cb = -1 - r
        return (content[cb // 4] >> (2 * (cb % 4))) & 3

    for j in S.jobs:
        twice = j.offset + sum(2 * j.in_w[q] * ref(j.in_ref[q]) for q in range(j.n_in))
        for f in range(j.n_out):
            if j.kind == F.JOB_SIGN:
                val[j.out_gate[f]] = int(twice > 0)
            else:
                assert twice % 2 == 0 and 0 <= twice // 2 < 16
                val[j.out_gate[f]] = j.lut[f][twice // 2]
    if S.out_gate < 0:
        return S.out_const
    return S.out_const + S.out_w * val[S.out_gate]


@pytest.mark.parametrize("content,pattern", [("xyabcz", "/abc/"), ("abcdef", CONFIG3), ("ab1def", CONFIG3),
                                             ("aabcdef", CONFIG5), ("aaadebcx", CONFIG5), ("In ThE end", "/the/i"),
                                             ("zzcdab", "/^(ab|cd)+/"), ("zzaXcz", "/a.c$/")])
def test_schedule_semantics(content, pattern):
    c = content.encode()
    S = F.schedule_match(len(c), pattern)
    assert S.level_off[0] == 0 and S.level_off[-1] == len(S.jobs)
    assert plain_schedule(S, c) == F.plain_match(c, pattern, engine=F.ENGINE_AUTO).result_lowered
    assert plain_schedule(S, c) == ro.has_match(content, pattern).result


def test_job_slices_partition():
    for J in (0, 1, 2, 7, 254, 512):
        for world in (1, 2, 3, 8):
            cover = []
            for r in range(world):
                a, b = F.job_slice(J, world, r)
                assert 0 <= a <= b <= J
                cover += list(range(a, b))
            assert cover == list(range(J))
            assert F.job_slice(J, world, 0)[1] >= 1 or J == 0  # rank 0 owns a lone job


@pytest.mark.parametrize("L,pattern,grammar", [(256, "/abc/", 0), (6, "/abc/", 0), (256, "/^[a-z0-9]+$/", 1),
                                               (1024, "/the/i", 0), (512, CONFIG5, 0), (40, "/^(ab|cd)+/", 0)])
def test_closure_parts(L, pattern, grammar):
    """Dependency-closure sharding: every rank's job set is closed under inputs,
    the frontier parts partition the jobs feeding the top, the top reads only
    top or frontier outputs, and the top holds the final output."""
    S = F.schedule_match(L, pattern, grammar=grammar)
    nl = len(S.level_off) - 1
    prod = {g: gi for gi, j in enumerate(S.jobs) for g in j.out_gate[:j.n_out]}

    def ids(runs_by_level):
        return {S.level_off[l] + i for l, rs in enumerate(runs_by_level) for a, b in rs for i in range(a, b)}

    for world in (1, 2, 3, 8):
        runs, frontier, top = F.closure_parts(S, world)
        T = ids(top)
        assert S.out_gate < 0 or prod[S.out_gate] in T
        fronts = [{S.level_off[l] + i for l, a, b in fr for i in range(a, b)} for fr in frontier]
        allfront = set().union(*fronts)
        assert sum(len(f) for f in fronts) == len(allfront)  # a partition
        for gi in T:
            j = S.jobs[gi]
            assert all(prod[j.in_ref[q]] in T | allfront for q in range(j.n_in) if j.in_ref[q] >= 0)
        for r in range(world):
            mine = ids(runs[r])
            assert fronts[r] <= mine  # (a widened top may also be an input of the frontier: run twice)
            for gi in mine:
                j = S.jobs[gi]
                assert all(prod[j.in_ref[q]] in mine for q in range(j.n_in) if j.in_ref[q] >= 0)
        if world > 1 and L >= 256:  # the split is balanced to within the edge jobs
            level0 = [sum(b - a for a, b in runs[r][0]) for r in range(world)]
            assert max(level0) <= 1.2 * (S.level_off[1] / world) + 8


class OracleShardExec:
    """run_sharded executor on the CPU oracle: LWE outputs of a schedule's jobs."""

    def __init__(self, O, S: F.Schedule, content_lwes: np.ndarray):
        self.O, self.S = O, S
        self.lwe_len = O.big + 1
        self.content = content_lwes.reshape(-1, self.lwe_len)
        self.levels = len(S.level_off) - 1
        self.val = {}

    def jobs(self, l):
        return self.S.level_off[l + 1] - self.S.level_off[l]

    def buffer_device(self):
        return torch.device("cpu")

    def _jobs(self, l, a, b):
        base = self.S.level_off[l]
        return self.S.jobs[base + a:base + b]

    def outputs(self, l, a, b):
        return sum(j.n_out for j in self._jobs(l, a, b))

    def run(self, l, a, b):
        rows, index, jobs = [], {}, []
        for j in self._jobs(l, a, b):
            ins = []
            for q in range(j.n_in):
                r = j.in_ref[q]
                if r not in index:
                    index[r] = len(rows)
                    rows.append(self.val[r] if r >= 0 else self.content[-1 - r])
                ins.append((index[r], j.in_w[q]))
            luts = [list(j.lut[f]) for f in range(j.n_out)]
            jobs.append((ins, j.offset, luts, j.kind))
        outs = self.O.gates(jobs, np.stack(rows))
        k = 0
        for j in self._jobs(l, a, b):
            for f in range(j.n_out):
                self.val[j.out_gate[f]] = outs[k]
                k += 1

    def export(self, l, a, b, cap):
        buf = np.zeros((max(cap, 1), self.lwe_len), dtype=np.uint64)
        k = 0
        for j in self._jobs(l, a, b):
            for f in range(j.n_out):
                buf[k] = self.val[j.out_gate[f]]
                k += 1
        return torch.from_numpy(buf.view(np.int64).reshape(-1))

    def import_(self, l, a, b, t):
        buf = t.numpy().view(np.uint64).reshape(-1, self.lwe_len)
        k = 0
        for j in self._jobs(l, a, b):
            for f in range(j.n_out):
                self.val[j.out_gate[f]] = buf[k].copy()
                k += 1

    def result(self) -> np.ndarray:
        S = self.S
        out = np.zeros(self.lwe_len, dtype=np.uint64)
        if S.out_gate >= 0:
            out = (np.uint64(S.out_w & 0xFFFFFFFFFFFFFFFF) * self.val[S.out_gate]).astype(np.uint64)
        out[-1] += np.uint64((S.out_const << 59) & 0xFFFFFFFFFFFFFFFF)
        return out


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle():
    import oracle_ffi as of
    return of.Oracle(of.load_fixture_key(), seed=SEED)


def _rank_main(rank: int, world: int, port: int, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        O = _oracle()
        got = []
        for i, (content, pattern) in enumerate(GLOO_CASES):
            c = content.encode()
            S = F.schedule_match(len(c), pattern)
            ex = OracleShardExec(O, S, O.encrypt_str(c, seed=100 + i))
            gathered = F.run_sharded(ex, world, rank, F.torch_all_gather())
            ex2 = OracleShardExec(O, S, O.encrypt_str(c, seed=100 + i))
            F.run_closure_sharded(ex2, S, world, rank, F.torch_all_gather())
            if rank == 0:
                got.append((ex.result(), gathered, ex2.result()))
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


def test_sharded_lwes_gloo():
    """World size 2, gloo: real LWEs all-gathered level by level (config 3 and
    config 5 patterns, anchored); result vs the plaintext oracle and vs the
    unsharded evaluation of the same schedule, bit for bit; dependency-closure
    sharding (one gather of the frontier) gives the same bits."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    O = _oracle()
    for i, ((content, pattern), (lwe, gathered, lwe_closure)) in enumerate(zip(GLOO_CASES, got)):
        want = ro.has_match(content, pattern).result
        assert int(O.decode16(lwe)[0]) == want, (content, pattern)
        S = F.schedule_match(len(content), pattern)
        assert gathered == sum(j.n_out for j in S.jobs[:S.level_off[-2]])  # every level but the last
        ex = OracleShardExec(O, S, O.encrypt_str(content.encode(), seed=100 + i))
        F.run_sharded(ex, 1, 0, lambda b: [b])
        assert np.array_equal(ex.result(), lwe)
        assert np.array_equal(lwe_closure, lwe)  # closure sharding: the same bits
    assert [ro.has_match(c, p).result for c, p in GLOO_CASES] == [1, 0, 1, 0]


CLOSURE4_CASES = [("xyabcz", "/abc/"), ("bcdefg", CONFIG3), ("aabcdef", CONFIG5)]


def _closure_rank_main(rank: int, world: int, port: int, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        O = _oracle()
        got = []
        for i, (content, pattern) in enumerate(CLOSURE4_CASES):
            c = content.encode()
            S = F.schedule_match(len(c), pattern)
            ex = OracleShardExec(O, S, O.encrypt_str(c, seed=200 + i))
            F.run_closure_sharded(ex, S, world, rank, F.torch_all_gather(), F.closure_parts(S, world))
            if rank == 0:
                got.append(ex.result())
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


def test_closure_sharded_gloo_world4():
    """World size 4, gloo: closure sharding with uneven parts (4, 3, 3, 3) and a
    top widened below the last level (short contents), real LWEs; bit-identical
    to the unsharded evaluation."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_closure_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    O = _oracle()
    for i, ((content, pattern), lwe) in enumerate(zip(CLOSURE4_CASES, got)):
        S = F.schedule_match(len(content), pattern)
        ex = OracleShardExec(O, S, O.encrypt_str(content.encode(), seed=200 + i))
        F.run_sharded(ex, 1, 0, lambda b: [b])
        assert np.array_equal(ex.result(), lwe), (content, pattern)
        assert int(O.decode16(lwe)[0]) == ro.has_match(content, pattern).result


# ------------------------------------------------------------------- GPU
def _two_rank_sharded(ctxs, content, pattern, seed):
    """Both 'ranks' on device 0: each runs its slices; the gather concatenates
    the exported device buffers (what all_gather_into_tensor does across GPUs)."""
    plans = []
    for ctx in ctxs:
        hs = ctx.upload_radix(ctx.encrypt_str(content, seed=seed))
        plans.append(F.ShardPlan(ctx, hs, pattern))
    world = len(ctxs)
    nl = plans[0].levels
    for l in range(nl - 1):
        parts = [F.job_slice(plans[0].jobs(l), world, r) for r in range(world)]
        counts = [plans[0].outputs(l, a, b) for a, b in parts]
        bufs = []
        for r, P in enumerate(plans):
            a, b = parts[r]
            if b > a:
                P.run(l, a, b)
            bufs.append(P.export(l, a, b, max(counts)))
        for r, P in enumerate(plans):
            for s, (a, b) in enumerate(parts):
                if s != r and counts[s]:
                    P.import_(l, a, b, bufs[s])
    plans[0].run(nl - 1, 0, plans[0].jobs(nl - 1))
    out, st = plans[0].finish()
    return plans, out, st


@pytest.mark.gpu
@pytest.mark.parametrize("content,pattern", [("bcdefghijklmnopq", CONFIG3), ("bcdefghijklmnoPq", CONFIG3),
                                             ("aaa" + "bcde" * 6 + "f", CONFIG5), ("xxxxxabcxxxxxxxxxxxx", "/abc/")])
def test_shard_plan_two_ranks_gpu(key_blob, content, pattern):
    ctxs = []
    for _ in range(2):
        ctx = F.Context(device=0)
        ctx.load_client_key(key_blob)
        ctx.gen_server_key(SEED)
        ctxs.append(ctx)
    plans, out, st = _two_rank_sharded(ctxs, content, pattern, seed=21)
    got = ctxs[0].download_radix(out)
    assert ctxs[0].decrypt_radix(got) == ro.has_match(content, pattern).result
    hs = ctxs[0].upload_radix(ctxs[0].encrypt_str(content, seed=21))
    ref, rst = ctxs[0].has_match(hs, pattern)
    assert np.array_equal(got, ctxs[0].download_radix(ref))  # bit-identical to the unsharded match
    assert (st.ct_ops, st.blind_rotations, st.levels) == (rst.ct_ops, rst.blind_rotations, rst.levels)
    for P in plans:
        P.free()


def _two_rank_closure(ctxs, content, pattern, seed):
    """run_closure_sharded with both 'ranks' on device 0: rank 1 runs its closure
    first and its frontier export stands in for the all_gather."""
    world = len(ctxs)
    S = F.schedule_match(len(content), pattern)
    plans = [F.ShardPlan(ctx, ctx.upload_radix(ctx.encrypt_str(content, seed=seed)), pattern) for ctx in ctxs]
    sent = {}

    for r in range(world - 1, -1, -1):
        def gather(buf, r=r):
            sent[r] = buf.clone()
            return [sent.get(q) for q in range(world)]
        F.run_closure_sharded(plans[r], S, world, r, gather)
    out, st = plans[0].finish()
    return plans, out, st


@pytest.mark.gpu
@pytest.mark.parametrize("content,pattern", [("bcdefghijklmnopq", CONFIG3), ("aaa" + "bcde" * 6 + "f", CONFIG5),
                                             ("xxxxxabcxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx", "/abc/"),
                                             ("x" * 40, "/abc/")])
def test_closure_two_ranks_gpu(key_blob, content, pattern):
    ctxs = []
    for _ in range(2):
        ctx = F.Context(device=0)
        ctx.load_client_key(key_blob)
        ctx.gen_server_key(SEED)
        ctxs.append(ctx)
    plans, out, st = _two_rank_closure(ctxs, content, pattern, seed=23)
    got = ctxs[0].download_radix(out)
    assert ctxs[0].decrypt_radix(got) == ro.has_match(content, pattern).result
    hs = ctxs[0].upload_radix(ctxs[0].encrypt_str(content, seed=23))
    ref, _ = ctxs[0].has_match(hs, pattern)
    assert np.array_equal(got, ctxs[0].download_radix(ref))  # bit-identical to the unsharded match
    for P in plans:
        P.free()


# ----------------------------------------------- full-size sharded parity (GPU)
def _config4(planted):
    """BASELINE config 4 content: 1024 letters/spaces without any case variant of
    'the', planted once at 700 (bench.py make_content 'letters')"""
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ ", dtype=np.uint8)
    s = bytearray(rng.choice(alpha, 1024))
    for i in range(len(s) - 2):
        if bytes(s[i:i + 3]).lower() == b"the":
            s[i + 2] = ord("x")
    if planted:
        s[700:703] = b"ThE"
    return s.decode()


def _config5(bad):
    import random
    r5 = random.Random(5)
    c = "aaa" + "".join(r5.choice(["bc", "de"]) for _ in range(254)) + "f"
    return c[:300] + "x" + c[301:] if bad else c


@pytest.fixture(scope="module")
def four_ctx(key_blob):
    """four contexts on device 0 standing in for four ranks"""
    ctxs = []
    for _ in range(4):
        ctx = F.Context(device=0)
        ctx.load_client_key(key_blob)
        ctx.gen_server_key(SEED)
        ctxs.append(ctx)
    return ctxs


FULL = [("config4-planted", "/the/i", lambda: _config4(True)), ("config4-absent", "/the/i", lambda: _config4(False)),
        ("config5", CONFIG5, lambda: _config5(False)), ("config5-bad", CONFIG5, lambda: _config5(True))]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["closure", "level"])
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name,pattern,make", FULL, ids=[f[0] for f in FULL])
def test_full_size_sharded_gpu(four_ctx, name, pattern, make, world, mode):
    """BASELINE configs 4 (/the/i, 1024 chars, planted and absent) and 5 (512 chars,
    merged engine) at their full sizes, split over 2 and 4 'ranks' (contexts on
    device 0) by closure and by level sharding (start offsets engine.rs:15-18,
    anchors engine.rs:51-57): the result is bit-identical to the unsharded
    fr_has_match and decrypts to the oracle's position-set simulator bit."""
    content = make()
    ctxs = four_ctx[:world]
    if mode == "closure":
        plans, out, st = _two_rank_closure(ctxs, content, pattern, seed=31)
    else:
        plans, out, st = _two_rank_sharded(ctxs, content, pattern, seed=31)
    got = ctxs[0].download_radix(out)
    exp = ro.has_match_reach(content, pattern)
    assert ctxs[0].decrypt_radix(got) == exp
    hs = ctxs[0].upload_radix(ctxs[0].encrypt_str(content, seed=31))
    ref, rst = ctxs[0].has_match(hs, pattern)
    assert np.array_equal(got, ctxs[0].download_radix(ref))  # bit-identical to the unsharded match
    assert (st.blind_rotations, st.levels) == (rst.blind_rotations, rst.levels)
    for P in plans:
        P.free()
    for h in hs + [ref, out]:
        ctxs[0].release(h)
