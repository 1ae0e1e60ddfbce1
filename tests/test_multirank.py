"""N>1 path on CPU: start-offset sharding over a world-size-2 gloo group.

Each rank evaluates its contiguous start-offset range (what fr_has_match_range
does on its GPU), the per-rank booleans are all-gathered and OR-reduced (what
bench.py does over RCCL followed by one threshold bootstrap on rank 0); the
result must equal the unsharded match.  Runs the product's plaintext semantics
(fr_plain_match, no GPU) so it covers the host-side shard logic only.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "fhe-regex_amd"))
import fheregex as F  # noqa: E402

CASES = [
    (b"xxxxxxxabcxxxxxxxx", "/abc/"),   # match inside rank 0's range
    (b"xxxxxxxxabcxxxxxxx", "/abc/"),   # match starting at the boundary (rank 1)
    (b"xxxxxxxabcxxxxxxx", "/abc/"),    # odd length, straddles the cut
    (b"xxxxxxxxxxxxxxxxx", "/abc/"),    # no match
    (b"abzzzzzzzzzzzzzzzz", "/^ab/"),   # anchored: only start 0 can match
    (b"zzzzzzzzzzzzzzzzab", "/ab$/"),
    (b"zzzzzzzzThEzzzzzzz", "/the/i"),
    (b"zzzzzzzcdabzzzzzzz", "/(ab|cd)+/"),
    (b"zzzzzzzzaXczzzzzzz", "/a.c/"),
]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank: int, world: int, port: int, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        got = []
        for content, pattern in CASES:
            lo, hi = F.shard_starts(len(content), world, rank)
            local = F.plain_match(content, pattern, start_lo=lo, start_hi=hi).result_lowered
            t = torch.tensor([local], dtype=torch.int64)
            parts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            got.append(int(any(int(p.item()) for p in parts)))
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_start_offset_shards_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [F.plain_match(c, p).result_lowered for c, p in CASES]
    assert got == want
    assert want == [1, 1, 1, 0, 1, 1, 1, 1, 1]


def test_shard_starts_partition():
    for L in (0, 1, 7, 256, 1023):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                lo, hi = F.shard_starts(L, world, r)
                assert 0 <= lo <= hi <= L
                covered += list(range(lo, hi))
            assert covered == list(range(L))


@pytest.mark.parametrize("pattern,reach", [("/abc/", 2), ("/the/i", 2), ("/a.c/", 2), ("/^ab/", 1)])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_content_window_covers_the_starts(pattern, reach, world):
    """fheregex.content_window (bench.py's start shards hold only this window): the
    characters a start range's circuit reads, from the lowered schedule -- for a
    fixed-width pattern, the starts themselves plus width - 1 characters, clipped at the
    end of the content (engine.rs:45-214: a branch reads the characters after its start)."""
    L = 256 * world
    for r in range(world):
        lo, hi = F.shard_starts(L, world, r)
        wlo, whi = F.content_window(L, pattern, lo, hi)
        if pattern.startswith("/^"):
            assert (wlo, whi) == ((0, reach + 1) if r == 0 else (lo, lo))  # anchored: start 0 only
            continue
        assert wlo == lo and whi == min(L, hi + reach), (r, wlo, whi)


def test_or_each_checks_group_sizes():
    """Context.or_each (the batched final bitor of start-sharded matches) takes 1..16
    booleans per group (one threshold gate each), refused before any device call."""
    ctx = F.Context(-1)
    with pytest.raises(ValueError):
        ctx.or_each([list(range(17))])
    with pytest.raises(ValueError):
        ctx.or_each([[]])
    assert ctx.or_each([]) == []
