"""Benchmark: TFHE gate-bootstraps/sec and end-to-end match time of /abc/ on
256-char content (BASELINE.json metric), on MI355X through the C-ABI.

One step = one homomorphic has_match of the workload's pattern over its
content (real encryptions under the reference's fixture client key, inputs
resident in HBM): parse -> enumerate -> record -> lower -> level-scheduled
KS + blind-rotation launches -> result (repeat matches replay the cached plan).

Workloads (--workload; BASELINE.json configs): metric = /abc/ on 256 printable
chars with "abc" at 200; config2 = /abc/ on 64 chars (run it with --params
k2n1024, BASELINE's "N=1024"); config3 = /^[a-z0-9]+$/ on 256 chars (grammar
extension: the reference returns Err); config4 = /the/i on 1024 chars;
config5 = /^a{2,8}(bc|de)+[^xyz]$/ on 512 chars (state-merging engine).

N > 1 (one process per GPU, torch.distributed over RCCL):
  --scaling strong (default): the named content length is fixed and ONE match
    is split across the ranks (fr_shard_* C-ABI).  --shard closure (default,
    fheregex.run_closure_sharded): the jobs feeding the top of the circuit are
    cut into contiguous parts, each rank runs the dependency closure of its part
    (the circuit is local in the content: a few edge jobs run on two ranks), one
    all_gather_into_tensor (RCCL, device to device) brings the parts' LWEs to
    rank 0, which runs the top.  --shard level (fheregex.run_sharded): each rank
    runs a contiguous slice of every level's jobs and every level's output LWEs
    are all-gathered.
  --scaling weak: --chars start offsets per GPU (content grows with N); each
    rank matches its start range on the content window those starts read, the
    per-rank booleans are all-gathered device to device and OR-ed on rank 0.

value = blind rotations executed by all ranks per second of wall time (one
rotation can serve several LUTs: multi-value bootstrapping; the LUT-output
rate is reported beside it, never as the value); ms_per_step = match time.
roofline: the blind-rotation kernel on rank 0, HIP events on the library's
stream over the timed region; algorithmic bytes per bootstrap
n*(k+1)^2*l*N*8; traffic / compute from the rocprofv3 PMC pass
of this kernel source (tools/profile.sh -> tools/pmc_summary.py).
cpu_baseline: the CPU restatement (oracle/, "port") timed on this host.
"""
import argparse
import hashlib
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
# measured wave64 v_fma_f64 issue: 54 lane-ops per CU-clock = 0.84 VALU wave-instructions
# per CU-clock (tools/ubench_f64.hip, profiles/r01/ubench_f64.log)
VALU_F64_PEAK = 54.0 / 64.0
SERVER_KEY_SEED = 42
CONFIG5 = "/^a{2,8}(bc|de)+[^xyz]$/"
WORKLOADS = {
    "metric": dict(pattern="/abc/", chars=256, content="printable"),
    "config2": dict(pattern="/abc/", chars=64, content="printable"),
    "config3": dict(pattern="/^[a-z0-9]+$/", chars=256, content="alnum", grammar=F.GRAMMAR_EXT),
    "config4": dict(pattern="/the/i", chars=1024, content="letters"),
    "config5": dict(pattern=CONFIG5, chars=512, content="config5"),
}


def algorithmic_bytes_per_pbs(p) -> int:
    # GGSW stream one bootstrap consumes: n * (k+1)^2 * level * N * 8 bytes
    return p.n * (p.k + 1) ** 2 * p.pbs_level * p.N * 8


def make_content(kind: str, L: int) -> bytes:
    """Seeded synthetic content of the workload (every workload matches)."""
    rng = np.random.default_rng(0)
    if kind == "printable":
        c = bytearray(rng.integers(0x20, 0x7F, L, dtype=np.uint8).tobytes())
        at = 200 if L >= 256 else L // 4
        c[at:at + 3] = b"abc"
        return bytes(c)
    if kind == "alnum":
        alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
        return bytes(rng.choice(alpha, L))
    if kind == "letters":  # /the/i planted once at 700 (or L*2/3), no other case variant of "the"
        alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ ", dtype=np.uint8)
        s = bytearray(rng.choice(alpha, L))
        for i in range(L - 2):
            if bytes(s[i:i + 3]).lower() == b"the":
                s[i + 2] = ord("x")
        at = 700 if L >= 1024 else (2 * L) // 3
        s[at:at + 3] = b"ThE"
        return bytes(s)
    if kind == "config5":  # a{3}(bc|de)*f: matches /^a{2,8}(bc|de)+[^xyz]$/ for even L
        import random
        r5 = random.Random(5)
        c = ("aaa" + "".join(r5.choice(["bc", "de"]) for _ in range((L - 4) // 2)) + "f").encode()
        assert len(c) == L, "config5 content needs an even length"
        return c
    raise ValueError(kind)


def content_window(L: int, pattern: str, lo: int, hi: int, grammar: int, engine: int, lowering: int):
    """[wlo, whi): the content positions the circuit of starts [lo, hi) reads
    (from the lowered schedule, so no --halo guess)."""
    S = F.schedule_match(L, pattern, lo, hi, lowering=lowering, engine=engine, grammar=grammar)
    pos = [(-1 - j.in_ref[q]) // 4 for j in S.jobs for q in range(j.n_in) if j.in_ref[q] < 0]
    return (min(pos), max(pos) + 1) if pos else (lo, lo)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(params, content: bytes, pattern: str, grammar: int, engine: int, lowering: int,
                 sample: int, match_max_jobs: int):
    """The oracle (oracle/: the CPU restatement of this path, test infrastructure)
    timed on this host: 1-thread and all-threads gate-bootstrap rates
    on a sample of eq-nibble gates, and the CPU end-to-end match of the workload on
    the same lowered schedule (the reference's serial fold, engine.rs:22-35)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_ffi as of

    O = of.Oracle(of.load_fixture_key(), seed=SERVER_KEY_SEED, k=params.k, N=params.N, ring=params.ring)
    threads = O.num_threads()
    lut = [int(v == 1) for v in range(16)]
    blocks = O.encrypt_blocks([i % 4 for i in range(2 * sample)], seed=5)
    gates = [([(2 * i, 1), (2 * i + 1, 4)], 0, lut) for i in range(sample)]
    O.set_threads(1)
    n1 = max(4, sample // 48)
    t0 = time.perf_counter()
    O.gates(gates[:n1], blocks)
    t1 = time.perf_counter() - t0
    O.set_threads(threads)
    t0 = time.perf_counter()
    O.gates(gates, blocks)
    tall = time.perf_counter() - t0
    rate_all = sample / tall
    S = F.schedule_match(len(content), pattern, lowering=lowering, engine=engine, grammar=grammar)
    match = {"jobs": len(S.jobs), "levels": len(S.level_off) - 1}
    if len(S.jobs) <= match_max_jobs:
        ct = O.encrypt_str(content, seed=7)
        t0 = time.perf_counter()
        res = O.run_schedule(S, ct)
        match["ms"] = (time.perf_counter() - t0) * 1e3
        match["result_decrypted"] = int(O.decode16(res)[0])
        match["how"] = "measured: every job of the lowered schedule on the CPU, level by level"
    else:
        match["ms"] = len(S.jobs) / rate_all * 1e3
        match["how"] = f"estimated: jobs / all-threads rate (more than {match_max_jobs} jobs)"
    ring = "f64 FFT" if params.ring == F.RING_FFT else "RNS NTT"
    return {
        "value": rate_all,
        "unit": "gate-bootstraps/s",
        "cores": threads,
        "kind": "port",
        "label": "build CPU restatement (oracle/, unoptimised, not tfhe-rs): a lower bound on a CPU path",
        "value_1t": n1 / t1,
        "value_all": rate_all,
        "nproc": os.cpu_count(),
        "model": cpu_model(),
        "match_ms": match["ms"],
        "match": match,
        "sample": f"{sample} eq-nibble gate bootstraps (lincomb+KS+BR+SE, k={params.k} N={params.N}, {ring} ring) "
                  f"on {threads} OpenMP threads in {tall:.1f} s; {n1} on 1 thread in {t1:.1f} s",
    }


def pmc_figures(params, path: str):
    """traffic (HBM bytes per BR launch) and the VALU issue rate of the BR kernel
    from tools/pmc_summary.py's JSON; stale when the kernel source changed since."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("ring", "rns") != ("fft" if params.ring == F.RING_FFT else "rns") or d.get("k", 1) != params.k:
        return None
    src = os.path.join(REPO, "fhe-regex_amd", "csrc", "fft_br.hip")
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16] if os.path.exists(src) else None
    return {"traffic": d.get("hbm_bytes_per_launch"), "valu_per_cu_clk": d.get("valu_per_cu_clk"),
            "source": os.path.relpath(path, REPO), "stale": d.get("kernel_sha") != sha}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="metric", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="N>1: strong = the workload's content split across ranks (one match, level-sharded); "
                         "weak = --chars start offsets per GPU")
    ap.add_argument("--shard", default="closure", choices=["closure", "level"],
                    help="strong scaling: closure = each rank runs the dependency closure of its part of the "
                         "circuit's top inputs, one gather of those to rank 0 (fheregex.run_closure_sharded); "
                         "level = every level split into job slices, all-gathered level by level")
    ap.add_argument("--chars", type=int, default=0, help="content chars (strong: total; weak: per GPU); 0: workload's")
    ap.add_argument("--pattern", default="", help="override the workload's pattern")
    ap.add_argument("--content", default="", choices=["", "printable", "alnum", "letters", "config5"])
    ap.add_argument("--params", default="k1n2048", choices=["k1n2048", "k2n1024"])
    ap.add_argument("--ring", default="auto", choices=["auto", "fft", "rns"])
    ap.add_argument("--engine", default="auto", choices=["auto", "enumerate", "merged"])
    ap.add_argument("--lowering", default="threshold", choices=["threshold", "faithful"])
    ap.add_argument("--cpu-sample", type=int, default=384, help="gates in the CPU baseline sample (0: skip)")
    ap.add_argument("--cpu-match-max-jobs", type=int, default=2000, help="largest schedule the CPU match runs")
    ap.add_argument("--saturate", type=int, default=2048, help="gates in the saturated throughput probe (0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 collectives (nccl = RCCL over xGMI; gloo only to rehearse ranks sharing one GPU)")
    ap.add_argument("--probe", default="", help="comma-separated batch sizes: blind-rotation ms per launch vs batch")
    ap.add_argument("--pmc", default="",
                    help="PMC summary of the BR kernel (tools/pmc_summary.py); default: profiles/r02/"
                         "pmc_summary.json at k1n2048, pmc_summary_k2n1024.json at k2n1024")
    args = ap.parse_args()
    if not args.pmc:
        args.pmc = os.path.join(REPO, "profiles", "r02",
                                "pmc_summary.json" if args.params == "k1n2048" else f"pmc_summary_{args.params}.json")

    W = WORKLOADS[args.workload]
    pattern = args.pattern or W["pattern"]
    kind = args.content or W["content"]
    grammar = W.get("grammar", F.GRAMMAR_REFERENCE)
    engine = {"auto": F.ENGINE_AUTO, "enumerate": F.ENGINE_ENUMERATE, "merged": F.ENGINE_MERGED}[args.engine]
    lowering = F.LOWER_THRESHOLD if args.lowering == "threshold" else F.LOWER_FAITHFUL

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    # one process per GPU; ranks beyond the visible devices (a gloo rehearsal on a
    # one-GPU box) share devices round-robin
    device = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        dist.init_process_group(args.dist_backend)
    coll_dev = torch.device("cuda", device) if args.dist_backend == "nccl" else torch.device("cpu")

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
    ctx.set_lowering(lowering)
    ctx.set_engine(engine)
    ctx.set_grammar(grammar)

    chars = args.chars or W["chars"]
    strong = args.scaling == "strong" or world == 1
    L = chars if strong else chars * world
    content = make_content(kind, L)
    expected = F.plain_match(content, pattern, engine=engine, grammar=grammar, lowering=lowering).result_lowered
    # content each rank holds: strong = all of it; weak = the window its starts read
    if strong:
        lo, hi, wlo, whi = 0, L, 0, L
    else:
        lo, hi = F.shard_starts(L, world, rank)
        wlo, whi = content_window(L, pattern, lo, hi, grammar, engine, lowering)
    handles = [F.NULL_CT] * L
    if whi > wlo:
        msgs = [(c >> (2 * b)) & 3 for c in content[wlo:whi] for b in range(4)]
        blocks = ctx.encrypt_blocks(msgs, seed=7, first_block=4 * wlo).reshape(whi - wlo, 4, ctx.lwe_len)
        for i, h in enumerate(ctx.upload_radix(blocks)):
            handles[wlo + i] = h

    plan = None
    if world > 1:
        gather = F.torch_all_gather()
        if strong:
            plan = F.ShardPlan(ctx, handles, pattern)
            sched = F.schedule_match(L, pattern, lowering=lowering, engine=engine, grammar=grammar)
            cparts = F.closure_parts(sched, world)  # once: the host derivation costs ms per call
            runs, _, top = cparts
            closure_rot = [sum(b - a for rl in runs[r] for a, b in rl) for r in range(world)]
            closure_rot[0] += sum(b - a for rl in top for a, b in rl)

    def step():
        """one match; returns (result handle on rank 0 or None, rotations run by this rank)"""
        if world == 1:
            out, st = ctx.has_match(handles, pattern)
            return out, st.blind_rotations, st
        if strong and args.shard == "closure":
            F.run_closure_sharded(plan, sched, world, rank, gather, cparts)
            if rank == 0:  # the match's rotations (jobs two ranks both ran count once)
                out, st = plan.finish()
                return out, len(sched.jobs), st
            return None, 0, plan.stats
        if strong:
            F.run_sharded(plan, world, rank, gather)
            mine = sum(len(range(*F.job_slice(plan.jobs(l), world, rank))) for l in range(plan.levels - 1))
            if rank == 0:
                out, st = plan.finish()
                return out, mine + plan.jobs(plan.levels - 1), st
            return None, mine, plan.stats
        out, st = ctx.has_match(handles, pattern, lo, hi)
        buf = torch.empty(ctx.lwe_len, dtype=torch.int64, device=f"cuda:{device}")
        ctx.export_bool_device([out], buf.data_ptr())
        ctx.release(out)
        recv = torch.cat(gather(buf))  # [world * lwe_len] on this GPU
        torch.cuda.synchronize()
        if rank != 0:
            return None, st.blind_rotations, st
        parts = ctx.import_bool_device(recv.data_ptr(), world)
        res = ctx.or_many(parts)
        for h in parts:
            ctx.release(h)
        return res, st.blind_rotations + (1 if world <= 15 else 2), st

    first_call = None
    for _ in range(args.warmup):
        o, _, st0 = step()
        if first_call is None:  # cold call: parse, record, lower, compile, plan upload
            first_call = {"host_ms": st0.host_ms, "device_ms": st0.device_ms, "plan_cached": st0.plan_cached}
        if o is not None:
            ctx.release(o)

    ctx.set_profiling(True)
    t_before = ctx.device_timers()
    barrier()
    t0 = time.perf_counter()
    rot_local = 0
    host_ms = 0.0
    out = None
    st = None
    for i in range(args.steps):
        o, rot, st = step()
        rot_local += rot
        host_ms += st.host_ms if world == 1 else 0.0
        if o is not None:
            if i + 1 < args.steps:
                ctx.release(o)
            else:
                out = o
    barrier()
    elapsed = time.perf_counter() - t0
    t_after = ctx.device_timers()
    ctx.set_profiling(False)

    if dist is not None:
        tt = torch.tensor([elapsed, float(rot_local)], dtype=torch.float64, device=coll_dev)
        mx = tt.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        elapsed, total_rot = float(mx[0]), float(tt[1])
    else:
        total_rot = float(rot_local)

    result = None
    if rank == 0:
        result = ctx.decrypt_radix(ctx.download_radix(out))
        if result != expected:
            print(f"WARNING: decrypted result {result} != expected {expected}", file=sys.stderr)

    kernel = None
    if args.saturate and rank == 0:
        src = [h for h in handles if h != F.NULL_CT]
        hs = [src[i % len(src)] for i in range(args.saturate)]
        br_sat, tot_sat = ctx.dev_bench_pbs(hs, 2)
        kernel = {"gates_per_launch": args.saturate, "br_ms_per_launch": br_sat / 2,
                  "pbs_per_s": 2 * args.saturate / (tot_sat / 1e3),
                  "br_pbs_per_s": 2 * args.saturate / (br_sat / 1e3)}

    probe = None
    if args.probe and rank == 0:
        src = [h for h in handles if h != F.NULL_CT]
        probe = {}
        for cnt in [int(x) for x in args.probe.split(",")]:
            hs = [src[i % len(src)] for i in range(cnt)]
            ctx.dev_bench_pbs(hs, 1)  # warm-up (the first launch of a shape runs on a cold clock)
            br_p, tot_p = ctx.dev_bench_pbs(hs, 2)
            probe[cnt] = {"br_ms": br_p / 2, "total_ms": tot_p / 2}

    if rank != 0:
        if plan is not None:
            plan.free()
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    bpp = algorithmic_bytes_per_pbs(params)
    br_ms = t_after["br_ms"] - t_before["br_ms"]
    br_launches = t_after["br_launches"] - t_before["br_launches"]
    br_gates = t_after["br_gates"] - t_before["br_gates"]
    achieved_gbs = (br_gates * bpp) / (br_ms / 1e3) / 1e9 if br_ms > 0 else 0.0
    pmc = pmc_figures(params, args.pmc)
    cpu = None
    if args.cpu_sample > 0 and world == 1:
        cpu = cpu_baseline(params, content, pattern, grammar, engine, lowering, args.cpu_sample,
                           args.cpu_match_max_jobs)
    ms_per_step = elapsed / args.steps * 1e3
    ring_name = "fft" if params.ring == F.RING_FFT else "rns"
    coll = "RCCL" if args.dist_backend == "nccl" else "gloo (host-staged)"
    if world == 1:
        par = "single GPU"
    elif strong and args.shard == "closure":
        par = (f"closure-sharded x{world} (each rank runs the dependency closure of its part of the top's inputs, "
               f"one {coll} all_gather of those LWEs, rank 0 runs the top)")
    elif strong:
        par = f"level-sharded x{world} (job slices per level, {coll} all_gather of each level's LWEs)"
    else:
        par = f"start-offset shards x{world} ({coll} all_gather of the per-rank booleans, OR on rank 0)"
    line = {
        "metric": METRIC,
        "value": total_rot / elapsed,
        "unit": "gate-bootstraps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: seeded content, real encryptions under the reference fixture client key",
        "config": {"workload": f"{args.workload}: {pattern} on {L} chars" + ("" if strong else f" ({chars} per GPU)"),
                   "content_chars": L, "params": args.params, "ring": ring_name, "lowering": args.lowering,
                   "engine": args.engine, "content": kind, "scaling": "strong" if strong else "weak",
                   "parallelism": par},
        "match_ms": ms_per_step,
        "blind_rotations_per_match": total_rot / args.steps,
        "lut_outputs_per_match": float(st.pbs) if world == 1 or strong else None,
        "levels": st.levels,
        "host_ms_per_match": host_ms / args.steps if world == 1 else None,
        "rotations_run_per_rank": closure_rot if world > 1 and strong and args.shard == "closure" else None,
        "first_call": first_call,
        "result_decrypted": result,
        "result_expected": expected,
        "keygen_s": t_key,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": pmc["traffic"] if pmc else None,
            "kernel": "k_blind_rotate_fft" if params.ring == F.RING_FFT else "k_blind_rotate",
            "achieved_is": "algorithmic GGSW bytes (n (k+1)^2 l N 8 per bootstrap) / average BR launch time",
            "bytes_per_pbs": bpp,
            "br_launches": br_launches,
            "br_avg_ms": br_ms / max(br_launches, 1),
            "br_gates_per_launch": br_gates / max(br_launches, 1),
            "compute": None if not pmc or pmc.get("valu_per_cu_clk") is None else {
                "bound": "valu",
                "achieved": pmc["valu_per_cu_clk"],
                "peak": VALU_F64_PEAK,
                "unit": "VALU wave-instructions per active-CU clock",
                "frac": pmc["valu_per_cu_clk"] / VALU_F64_PEAK,
                "peak_is": "measured wave64 v_fma_f64 issue rate (profiles/r01/ubench_f64.log)",
            },
            "pmc_source": pmc["source"] if pmc else None,
            "pmc_stale": pmc["stale"] if pmc else None,
        },
        "kernel_saturated": kernel,
        "latency_probe": probe,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    if plan is not None:
        plan.free()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
