"""Benchmark: TFHE gate-bootstraps/sec and end-to-end match time of /abc/ on
256-char content (BASELINE.json metric), on MI355X through the C-ABI.

One step = one homomorphic has_match of /abc/ over the rank's 256-char shard of
synthetic printable-ASCII content (real encryptions under the reference's fixture
client key, "abc" planted at global position 200): parse -> enumerate ->
record -> lower -> level-scheduled KS + blind-rotation launches -> result.
Ranks shard start offsets (weak scaling: 256 starts per GPU); for N > 1 the
per-rank boolean results are all-gathered over RCCL and OR-reduced with one
threshold bootstrap on rank 0 (inside the timed step).

value = gate bootstraps (blind rotations) executed by all ranks per second of
wall time (multi-value bootstrapping lets one rotation serve several LUTs: the
LUT-output rate is reported beside it, never as the value);
ms_per_step = end-to-end match time.  roofline: blind-rotation kernel, HIP
events on the library's stream over the timed region, algorithmic bytes per
bootstrap n*(k+1)^2*l*N*8.  cpu_baseline: the CPU restatement
(oracle/, "port") timed on this host on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))

import numpy as np  # noqa: E402

import fheregex as F  # noqa: E402

METRIC = "TFHE gate-bootstraps/sec; end-to-end match time for /abc/ on 256-char content"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SERVER_KEY_SEED = 42


def algorithmic_bytes_per_pbs(p) -> int:
    # GGSW stream one bootstrap consumes: n * (k+1)^2 * level * N * 8 bytes
    return p.n * (p.k + 1) ** 2 * p.pbs_level * p.N * 8


def cpu_baseline(params_name: str, sample: int, ring: int):
    """Time the oracle (CPU restatement, test infrastructure) on this host, on
    the same ring as the GPU run."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_ffi as of

    key = of.load_fixture_key()
    k, N = (1, 2048) if params_name == "k1n2048" else (2, 1024)
    O = of.Oracle(key, seed=SERVER_KEY_SEED, k=k, N=N, ring=ring)
    threads = of.lib().or_num_threads()
    blocks = O.encrypt_blocks([i % 4 for i in range(2 * sample)], seed=5)
    lut = [int(v == 1) for v in range(16)]
    gates = [([(2 * i, 1), (2 * i + 1, 4)], 0, lut) for i in range(sample)]
    t0 = time.perf_counter()
    O.gates(gates, blocks)
    dt = time.perf_counter() - t0
    return {
        "value": sample / dt,
        "unit": "gate-bootstraps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample} eq-nibble gate bootstraps (lincomb+KS+BR+SE, {params_name}, "
                  f"{'f64 FFT' if ring == of.RING_FFT else 'RNS NTT'} ring) on the fixture key, "
                  f"{threads} OpenMP threads, {dt:.1f} s",
    }


def load_traffic(path):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), d
    except (OSError, ValueError):
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chars", type=int, default=256, help="content chars (start offsets) per GPU")
    ap.add_argument("--pattern", default="/abc/")
    ap.add_argument("--params", default="k1n2048", choices=["k1n2048", "k2n1024"])
    ap.add_argument("--ring", default="auto", choices=["auto", "fft", "rns"],
                    help="blind-rotation ring: f64-FFT torus (default for k1n2048) or the RNS NTT ring")
    ap.add_argument("--engine", default="auto", choices=["auto", "enumerate", "merged"],
                    help="regex evaluation: the reference's enumeration, state merging, or auto")
    ap.add_argument("--content", default="printable", choices=["printable", "config5"],
                    help="printable: seeded ASCII with 'abc' at 200; config5: a{3}(bc|de)*f (BASELINE config 5)")
    ap.add_argument("--lowering", default="threshold", choices=["threshold", "faithful"])
    ap.add_argument("--cpu-sample", type=int, default=384, help="gate bootstraps in the CPU baseline sample (0: skip)")
    ap.add_argument("--saturate", type=int, default=2048, help="gates in the saturated kernel-throughput probe (0: skip)")
    ap.add_argument("--halo", type=int, default=2, help="chars read past the last start (pattern span - 1; 2 for /abc/)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N>1 (nccl = RCCL over xGMI; gloo only to rehearse several ranks on one GPU)")
    ap.add_argument("--probe", default="", help="comma-separated batch sizes: blind-rotation ms per launch vs batch")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    # one process per GPU; ranks beyond the visible devices (a gloo rehearsal on
    # a one-GPU box) share devices round-robin
    device = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        dist.init_process_group(args.dist_backend)
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    k, N = (1, 2048) if args.params == "k1n2048" else (2, 1024)
    params = F.default_params(k=k, N=N, ring={"auto": None, "fft": F.RING_FFT, "rns": F.RING_RNS}[args.ring])
    with open(os.path.join(REPO, "tests", "golden", "client_key"), "rb") as f:
        blob = f.read()
    ctx = F.Context(device, params)
    ctx.load_client_key(blob)
    t_key = time.perf_counter()
    ctx.gen_server_key(SERVER_KEY_SEED)  # same seed on every rank: identical keys, no broadcast needed
    t_key = time.perf_counter() - t_key
    ctx.set_lowering(F.LOWER_THRESHOLD if args.lowering == "threshold" else F.LOWER_FAITHFUL)
    ctx.set_engine({"auto": F.ENGINE_AUTO, "enumerate": F.ENGINE_ENUMERATE, "merged": F.ENGINE_MERGED}[args.engine])

    # synthetic content: printable ASCII, "abc" planted at global position 200
    L = args.chars * world
    rng = np.random.default_rng(0)
    content = bytearray(rng.integers(0x20, 0x7F, L, dtype=np.uint8).tobytes())
    content[200:203] = b"abc"
    content = bytes(content)
    if args.content == "config5":  # matches /^a{2,8}(bc|de)+[^xyz]$/ when L is even
        import random
        r5 = random.Random(5)
        content = ("aaa" + "".join(r5.choice(["bc", "de"]) for _ in range((L - 4) // 2)) + "f").encode()
        assert len(content) == L, "config5 content needs an even length"
        args.halo = L  # anchored pattern: a branch reads to the end of the content
    lo, hi = F.shard_starts(L, world, rank)  # this rank's start offsets
    win_hi = min(L, hi + args.halo)          # + halo: chars a branch may read past its start
    msgs = [(c >> (2 * b)) & 3 for c in content[lo:win_hi] for b in range(4)]
    blocks = ctx.encrypt_blocks(msgs, seed=7, first_block=4 * lo).reshape(win_hi - lo, 4, ctx.lwe_len)
    handles = [F.NULL_CT] * L
    for i, h in enumerate(ctx.upload_radix(blocks)):
        handles[lo + i] = h

    def step():
        out, st = ctx.has_match(handles, args.pattern, lo, hi)
        final_pbs = 0
        if world > 1:
            lwe = ctx.download_radix(out)[0]
            t = torch.from_numpy(lwe.view(np.int64)).to(coll_dev)
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            if rank == 0:
                arr = np.stack([p.cpu().numpy().view(np.uint64) for p in parts])
                bh = ctx.upload_bool(arr)
                res = ctx.or_many(bh)
                final_pbs = 1 if world <= 15 else -1
                for h in bh:
                    ctx.release(h)
                ctx.release(out)
                out = res
        return out, st, final_pbs

    first_call = None
    for _ in range(args.warmup):
        o, st0, _ = step()
        if first_call is None:  # cold call: parse, record, lower, compile, plan upload
            first_call = {"host_ms": st0.host_ms, "device_ms": st0.device_ms, "plan_cached": st0.plan_cached}
        ctx.release(o)

    ctx.set_profiling(True)
    barrier()
    t0 = time.perf_counter()
    pbs_local = 0
    rot_local = 0
    br_ms = 0.0
    br_launches = 0
    br_gates = 0
    host_ms = 0.0
    levels = 0
    final_pbs_total = 0
    out = None
    for i in range(args.steps):
        o, st, fp = step()
        pbs_local += st.pbs
        rot_local += st.blind_rotations
        br_ms += st.br_kernel_ms
        br_launches += st.br_launches
        br_gates += st.br_gates
        host_ms += st.host_ms
        levels = st.levels
        final_pbs_total += max(fp, 0)
        if i + 1 < args.steps:
            ctx.release(o)
        else:
            out = o
    barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)

    if dist is not None:
        tt = torch.tensor([elapsed, float(pbs_local + final_pbs_total), float(rot_local + final_pbs_total)],
                          dtype=torch.float64, device=coll_dev)
        mx = tt.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        elapsed, total_pbs, total_rot = float(mx[0]), float(tt[1]), float(tt[2])
    else:
        total_pbs = float(pbs_local + final_pbs_total)
        total_rot = float(rot_local + final_pbs_total)

    result = None
    if rank == 0:
        result = ctx.decrypt_radix(ctx.download_radix(out))
        expected = 1 if 200 < L - 2 else 0
        if result != expected:
            print(f"WARNING: decrypted result {result} != expected {expected}", file=sys.stderr)

    # saturated kernel-throughput probe: one big batch of independent PBS
    kernel = None
    if args.saturate and rank == 0:
        hs = [handles[lo + (i % (win_hi - lo))] for i in range(args.saturate)]
        br_sat, tot_sat = ctx.dev_bench_pbs(hs, 2)
        kernel = {"gates_per_launch": args.saturate, "br_ms_per_launch": br_sat / 2,
                  "pbs_per_s": 2 * args.saturate / (tot_sat / 1e3),
                  "br_pbs_per_s": 2 * args.saturate / (br_sat / 1e3)}

    probe = None
    if args.probe and rank == 0:
        probe = {}
        for cnt in [int(x) for x in args.probe.split(",")]:
            hs = [handles[lo + (i % (win_hi - lo))] for i in range(cnt)]
            br_p, tot_p = ctx.dev_bench_pbs(hs, 2)
            probe[cnt] = {"br_ms": br_p / 2, "total_ms": tot_p / 2}

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    bpp = algorithmic_bytes_per_pbs(params)
    achieved_gbs = (br_gates * bpp) / (br_ms / 1e3) / 1e9 if br_ms > 0 else 0.0
    traffic, tinfo = load_traffic(os.path.join(REPO, "profiles", "r01", "pmc_summary.json"))
    if tinfo is not None and tinfo.get("ring", "rns") != ("fft" if params.ring == F.RING_FFT else "rns"):
        traffic = None  # the PMC summary was measured on the other ring
    cpu = cpu_baseline(args.params, args.cpu_sample, params.ring) if args.cpu_sample > 0 and world == 1 else None
    ms_per_step = elapsed / args.steps * 1e3
    ring_name = "fft" if params.ring == F.RING_FFT else "rns"
    line = {
        "metric": METRIC,
        "value": total_rot / elapsed,
        "unit": "gate-bootstraps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: seeded printable ASCII, real encryptions under the reference fixture client key",
        "config": {"workload": f"{args.pattern} contains-match, {args.chars} chars per GPU (start-offset shards)",
                   "content_chars": L, "params": args.params, "ring": ring_name, "lowering": args.lowering,
                   "engine": args.engine,
                   "content": args.content,
                   "parallelism": f"start-offset shards x{world}"},
        "match_ms": ms_per_step,
        "blind_rotations_per_match": total_rot / args.steps,
        "lut_outputs_per_match": total_pbs / args.steps,
        "lut_outputs_per_s": total_pbs / elapsed,
        "levels": levels,
        "host_ms_per_match": host_ms / args.steps,
        "first_call": first_call,
        "result_decrypted": result,
        "keygen_s": t_key,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": "k_blind_rotate_fft" if params.ring == F.RING_FFT else "k_blind_rotate",
            "bytes_per_pbs": bpp,
            "br_launches": br_launches,
            "br_avg_ms": br_ms / max(br_launches, 1),
            "br_gates_per_launch": br_gates / max(br_launches, 1),
        },
        "kernel_saturated": kernel,
        "latency_probe": probe,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
