"""Benchmark: TFHE gate-bootstraps/sec and end-to-end match time of /abc/ on
256-char content (BASELINE.json metric), on MI355X through the C-ABI.

One step = one homomorphic has_match of the workload's pattern over its
content (real encryptions under the reference's fixture client key, inputs
resident in HBM): parse -> enumerate -> record -> lower -> level-scheduled
KS + blind-rotation launches -> result (repeat matches replay the cached plan;
`fresh_content` times matches on newly encrypted content, which replay the same
template plan with the new slots bound).  --matches M: each step is M matches of
the pattern over M contents in shared launches (fr_has_match_batch).

Workloads (--workload; BASELINE.json configs): metric = /abc/ on 256 printable
chars with "abc" at 200; config2 = /abc/ on 64 chars (run it with --params
k2n1024, BASELINE's "N=1024"); config3 = /^[a-z0-9]+$/ on 256 chars (grammar
extension: the reference returns Err); config4 = /the/i on 1024 chars;
config5 = /^a{2,8}(bc|de)+[^xyz]$/ on 512 chars (state-merging engine).

N > 1 (one process per GPU, torch.distributed over RCCL).  `--gpus N` with no
WORLD_SIZE in the environment starts the N rank processes itself (a child
`python -m torch.distributed.run`, before anything touches the GPU) and exits with
their status; under an external launcher WORLD_SIZE must equal --gpus.
  --scaling weak (default): per-GPU work fixed.  --shard starts (default; BASELINE
    north_star's per-start-offset variants with a final bitor over RCCL): the content
    is --chars per GPU (the workload's length by default, so N x 256 chars for the
    metric), rank r owns start offsets [r chars, (r+1) chars) and holds only the
    content window those starts read; each rank matches its start range as up to
    16 // N booleans (fr_has_match_parts: its OR tree stops where the ranks' one threshold
    OR takes over; --start-parts 1: fr_has_match_range's single boolean), the booleans are
    all-gathered device to device and OR-ed on rank 0 (the reference's ct_or fold,
    engine.rs:22-35).  The
    same run also times weak scaling by matches (every rank its own full-length
    match, no data-path collective) into `weak_matches`, never `value`.
    --shard matches makes that the timed mode.
  --scaling strong: the named content length is fixed and ONE match is split
    across the ranks (fr_shard_* C-ABI; --shard starts: its start offsets, each rank
    matching its range on its window, the same gather and OR as the weak mode).  --shard closure (default,
    fheregex.run_closure_sharded): the jobs feeding the top of the circuit are
    cut into contiguous parts, each rank runs the dependency closure of its part,
    one all_gather_into_tensor (RCCL, device to device) brings the parts' LWEs to
    rank 0, which runs the top.  --shard level (fheregex.run_sharded): each rank
    runs a contiguous slice of every level's jobs and every level's output LWEs
    are all-gathered.  Per-rank phase times are in `per_rank`.  The circuit's four
    dependent levels bound this mode.

value = blind rotations executed by all ranks per second of wall time (one
rotation can serve several LUTs: multi-value bootstrapping; the LUT-output
rate is reported beside it, never as the value); ms_per_step = step time.
roofline: the blind-rotation kernel on rank 0, HIP events on the library's
stream over the timed region.  The kernel is VALU-bound (f64 FFT): `achieved` =
algorithmic f64 FLOP per bootstrap (algorithmic_flops_per_pbs) x bootstraps /
BR time against the FP64 vector peak; the HBM side reports the physical traffic
(rocprofv3 PMC of this kernel source, tools/profile.sh -> tools/pmc_summary.py)
per launch time.  cpu_baseline: the CPU restatement (oracle/, "port") timed on
this host's available cores.  kernel_saturated: 2048 bootstraps per launch, 10 launches
after a warm-up.  power: socket power and energy per bootstrap of rank 0's GPU over the
timed region and the saturated probe (the driver's energy accumulator, read outside
each region; --no-power skips it), against the board's power cap.
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "fhe-regex_amd"))
# hardware queues per process (read at HIP init): the `inflight_1ctx` record's lanes are
# streams of one context, and with HIP's default of 4 two of four lanes share a queue and
# serialise (tools/lanes_probe.py: 4 lanes 5.44 ms per match with 4 queues, 4.22 with 8); the
# timed single-stream match is unaffected
try:
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
except ValueError:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402

import fheregex as F  # noqa: E402

METRIC = "TFHE gate-bootstraps/sec; end-to-end match time for /abc/ on 256-char content"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec: 256 CUs x 128 FLOP/clk x 2.4 GHz
# wave64 f64 VALU instructions per CU-clock: spec 1.0 (4 SIMDs x 16 f64 lanes); measured
# v_fma_f64 issue 54 lane-ops per CU-clock = 0.84 (tools/ubench_f64.hip, profiles/r01/ubench_f64.log)
VALU_SPEC_PER_CU_CLK = 1.0
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


def algorithmic_flops_per_pbs(p) -> int:
    """f64 FLOP of one blind rotation on the FFT ring: ceil(n/2)
    unrolled steps, each 2(k+1) complex FFTs of M = N/2 points at 5 M log2 M and
    the external products with three Fourier GGSWs, (k+1)^2 complex MACs (8 FLOP)
    per GGSW and slot."""
    M = p.N // 2
    per_step = 2 * (p.k + 1) * 5 * M * (M.bit_length() - 1) + 3 * (p.k + 1) ** 2 * 8 * M
    return ((p.n + 1) // 2) * per_step


def available_cores():
    """CPU threads this process may use: the affinity mask, capped by the cgroup
    CPU quota and by OMP_NUM_THREADS (the GPU box sets it to its per-GPU CPU share)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    caps = {"affinity": aff, "cgroup_quota": quota, "omp_num_threads": omp}
    n = min(x for x in (aff, quota, omp) if x)
    why = [k for k, v in caps.items() if v == n]
    return n, dict(caps, capped_by=why[0] if why else "affinity")


def make_content(kind: str, L: int, seed: int = 0) -> bytes:
    """Seeded synthetic content of the workload (every workload matches)."""
    rng = np.random.default_rng(seed)
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
        r5 = random.Random(5 + seed)
        c = ("aaa" + "".join(r5.choice(["bc", "de"]) for _ in range((L - 4) // 2)) + "f").encode()
        assert len(c) == L, "config5 content needs an even length"
        return c
    raise ValueError(kind)


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
                 sample: int, match_max_jobs: int, content_lwes=None, gpu_words=None):
    """The oracle (oracle/: the CPU restatement of this path, test infrastructure)
    timed on this host: 1-thread and all-threads gate-bootstrap rates
    on a sample of eq-nibble gates, and the CPU end-to-end match of the workload on
    the same lowered schedule (the reference's serial fold, engine.rs:22-35).  With
    the GPU's content LWEs and result words, the CPU match runs on those very LWEs
    and `cpu_gpu_bit_identical` says whether its result equals the GPU's word for
    word."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_ffi as of

    O = of.Oracle(of.load_fixture_key(), seed=SERVER_KEY_SEED, k=params.k, N=params.N, ring=params.ring)
    threads, caps = available_cores()
    O.set_threads(threads)
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
    identical = None
    if len(S.jobs) <= match_max_jobs:
        ct = content_lwes if content_lwes is not None else O.encrypt_str(content, seed=7)
        t0 = time.perf_counter()
        res = O.run_schedule(S, ct)
        match["ms"] = (time.perf_counter() - t0) * 1e3
        match["result_decrypted"] = int(O.decode16(res)[0])
        match["how"] = "measured: every job of the lowered schedule on the CPU, level by level"
        if gpu_words is not None and content_lwes is not None:
            identical = bool(np.array_equal(np.asarray(gpu_words, dtype=np.uint64), res))
            match["inputs"] = "the GPU run's content LWEs (same server-key seed)"
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
        "cores_available": caps,
        "cores_note": f"all available threads: min(affinity, cgroup quota, OMP_NUM_THREADS) = {threads}, "
                      f"capped by {caps['capped_by']}",
        "model": cpu_model(),
        "match_ms": match["ms"],
        "match": match,
        "cpu_gpu_bit_identical": identical,
        "sample": f"{sample} eq-nibble gate bootstraps (lincomb+KS+BR+SE, k={params.k} N={params.N}, {ring} ring) "
                  f"on {threads} OpenMP threads in {tall:.1f} s; {n1} on 1 thread in {t1:.1f} s",
    }


def kernel_source_sha():
    """what the blind-rotation kernels are compiled from: fft_br.hip, the pair shape's translation
    unit and the Makefile that sets its scheduler (tools/pmc_summary.py hashes the same)"""
    h = hashlib.sha256()
    for rel in ("csrc/fft_br.hip", "csrc/fft_br_pair.hip", "Makefile"):
        path = os.path.join(REPO, "fhe-regex_amd", rel)
        if not os.path.exists(path):
            return None
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


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
    sha = kernel_source_sha()
    shapes = {}
    lns = d.get("launches", [])
    sat_grid = max((ln.get("grid", 0) for ln in lns), default=None)  # the saturated probe (as pmc_summary.py)
    for ln in lns:
        if ln.get("grid") == sat_grid:
            continue
        m = re.search(r"<\s*\d+,\s*\d+,\s*\d+,\s*(true|false),\s*(\d+)\s*>", ln.get("kernel", ""))
        if not m or not ln.get("calls"):
            continue
        shape = "throughput" if m.group(1) == "false" else ("pair" if m.group(2) == "2" else "latency")
        b, c = shapes.get(shape, (0.0, 0))
        shapes[shape] = (b + ln["hbm_bytes"] * ln["calls"], c + ln["calls"])
    return {"traffic": d.get("hbm_bytes_per_launch"), "valu_per_cu_clk": d.get("valu_per_cu_clk"),
            "traffic_per_shape": {k: b / c for k, (b, c) in shapes.items()},
            "source": os.path.relpath(path, REPO), "stale": d.get("kernel_sha") != sha}


def named_length_record(value, ms, L, named, M, world, strong, ok, strong_starts, steps):
    """BASELINE's named length (W["chars"]: 256 for the metric, 1,024 for config 4) at this N:
    `value` itself when its timed region is one match of that length (N = 1, or a strong
    split), else the strong_starts record (N > 1 with weak start shards: the named length
    split by start offsets); None when neither ran.  A 1 -> N scaling plot of the named
    workload reads named_length.value; `value` at N > 1 may be weak (N x the chars)."""
    if L == named and M == 1 and (world == 1 or strong):
        return {"chars": L, "value": value, "ms_per_step": ms, "steps": steps, "results_ok_steps": bool(ok),
                "source": "value"}
    if strong_starts and "value" in strong_starts:
        return {"chars": strong_starts["content_chars"], "value": strong_starts["value"],
                "ms_per_step": strong_starts["ms_per_step"], "steps": strong_starts["steps"],
                "results_ok_steps": strong_starts["results_ok_steps"], "source": "strong_starts"}
    return None


def north_star_hbm(per_shape):
    """north_star's ">= 50% HBM roofline on the external-product kernel", evaluated at the
    dominant launch shape (the most BR time in the timed region): the physical fraction
    (PMC bytes per launch / launch time) decides it; the algorithmic one (48.6 MB of GGSW per
    bootstrap) is a normalisation that counts the L2-shared key once per bootstrap"""
    live = {k: v for k, v in per_shape.items() if v}
    if not live:
        return None
    name, sh = max(live.items(), key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])
    phys = sh.get("hbm_physical_frac")
    return {"target": 0.5, "shape": name, "physical_frac": phys, "algorithmic_frac": sh["hbm_algorithmic_frac"],
            "met": bool(phys is not None and phys >= 0.5),
            "bound": "valu/LDS exchanges (f64 FFT butterflies and the transforms' LDS exchanges and barriers; the "
                     "key stream is shared through each XCD's L2, so HBM is not the bound)",
            "note": "target not met and not the bound: physical HBM traffic is a few percent of 8 TB/s; the "
                    "algorithmic figure is not a physical rate (it exceeds 1.0 at >= 512 bootstraps per launch)"}


class EnergyMeter:
    """Socket energy of this rank's GPU from the driver's energy accumulator (amdsmi; no HIP),
    read outside the timed regions: average power and energy per bootstrap of a region, and the
    board's power cap (tools/power_probe.py samples the same table every 4 ms).  Any failure
    (no amdsmi, no permission, no matching device) leaves the meter off: the records are null."""

    def __init__(self, torch_props):
        self.h = None
        self.cap_w = None
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            want = (torch_props.pci_domain_id, torch_props.pci_bus_id, torch_props.pci_device_id)
            for h in amdsmi.amdsmi_get_processor_handles():
                dom, bus, rest = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")
                if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                    self.h = h
            import atexit

            atexit.register(amdsmi.amdsmi_shut_down)
            if self.h is not None:
                self.amdsmi = amdsmi
                self.cap_w = amdsmi.amdsmi_get_power_cap_info(self.h)["power_cap"] / 1e6
        except Exception:  # noqa: BLE001 -- the meter is an extra, never a failure of the bench
            self.h = None

    def read(self):
        if self.h is None:
            return None
        try:
            e = self.amdsmi.amdsmi_get_energy_count(self.h)
            return e["energy_accumulator"] * e["counter_resolution"] * 1e-6, time.perf_counter()
        except Exception:  # noqa: BLE001
            return None

    def region(self, r0, r1, bootstraps):
        if r0 is None or r1 is None or r1[1] <= r0[1] or r1[0] < r0[0]:
            return None
        j, s = r1[0] - r0[0], r1[1] - r0[1]
        return {"w": j / s, "seconds": s, "mj_per_bootstrap": 1e3 * j / bootstraps if bootstraps else None}


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int, argv, job_timeout: float = 0.0, script: str = "") -> int:
    """`--gpus N` without a launcher: start N rank processes of this script with
    torch.distributed.run on 127.0.0.1 (one per GPU) and return their exit status.
    The caller has touched no GPU (no HIP call, no torch.cuda query) and never
    re-execs: the ranks are children.  job_timeout > 0: after that many seconds the
    launcher's whole process group is killed and 124 returned (a stuck rank or
    collective ends the job with a message instead of holding the node)."""
    import signal
    import threading

    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), script or os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver (RCCL)
    # the ranks' stdout: the JSON line passes, anything else (launcher / gloo chatter) goes to stderr
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1, start_new_session=True)
    expired = threading.Event()

    def kill_job():
        """the launcher and every process under it (torch.distributed.run starts each rank
        in a process group of its own, so the launcher's group alone misses them)"""
        expired.set()
        print(f"bench.py: the {n} ranks did not finish within --job-timeout {job_timeout:.0f} s; "
              f"killing the launcher and its ranks", file=sys.stderr, flush=True)
        try:
            import psutil

            tree = psutil.Process(proc.pid).children(recursive=True)
        except Exception:  # psutil absent or the launcher gone: its own group below
            tree = []
        for p in tree:
            try:
                p.kill()
            except Exception:
                pass
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass

    timer = threading.Timer(job_timeout, kill_job) if job_timeout > 0 else None
    if timer is not None:
        timer.daemon = True
        timer.start()
    for line in proc.stdout:
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    rc = proc.wait()
    if timer is not None:
        timer.cancel()
    return 124 if expired.is_set() else rc


def spawn_probe(world: int, rank: int):
    """--spawn-probe: the rank processes meet over gloo and report, without a GPU
    (the CPU test of the launcher path)."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
        mine = torch.tensor([rank, os.getpid(), os.getppid()], dtype=torch.int64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        rows = [v.tolist() for v in allr]
        dist.destroy_process_group()
    else:
        rows = [[0, os.getpid(), os.getppid()]]
    if rank == 0:
        print(json.dumps({"spawn_probe": True, "n_gpus": world, "ranks": [r[0] for r in rows],
                          "pids": [r[1] for r in rows], "parent_pids": [r[2] for r in rows]}))


# N > 1 default (scaling, shard) per workload: the metric (and config 2) grows the content
# with N, split by start offsets (weak); config 4 is BASELINE's "1024-char content, start
# offsets sharded across 8 GPUs", so its value is the named length split by start offsets
# (strong); the anchored configs 3 and 5 have one start, so one match is split by its
# dependency closures (strong)
N_GT_1_DEFAULT = {"metric": ("weak", "starts"), "config2": ("weak", "starts"), "config3": ("strong", "closure"),
                  "config4": ("strong", "starts"), "config5": ("strong", "closure")}


def default_mode(workload: str, scaling: str, shard: str):
    """--scaling / --shard as given, or the workload's N > 1 default where left empty"""
    ds, dsh = N_GT_1_DEFAULT[workload]
    if not scaling:
        scaling = ds
        if not shard and scaling == ds:
            shard = dsh
    return scaling, shard


def nccl_device_guard(backend: str, local_world: int, n_devices: int):
    """RCCL (like NCCL) refuses two ranks on one device: under nccl every local rank
    needs its own GPU.  Returns an error message, or None."""
    if backend == "nccl" and local_world > n_devices:
        return (f"--dist-backend nccl needs one GPU per rank: {local_world} local rank(s) but "
                f"{n_devices} visible device(s) (use --dist-backend gloo to rehearse ranks sharing a GPU)")
    return None


def resolve_mode(scaling: str, shard: str, world: int, matches: int, group1: bool = False):
    """(strong, shard) of a run: one GPU runs the plain (or batched) match; N > 1 weak
    defaults to start-offset shards, strong to closure sharding.  group1 (--one-rank-group):
    N = 1 runs the N > 1 start-shard pipeline over a one-rank process group."""
    scaling = scaling or "weak"
    strong = scaling == "strong" and world > 1
    shard = shard or ("closure" if strong else "starts")
    if world == 1 and group1:
        if shard != "starts" or matches != 1:
            raise ValueError("--one-rank-group runs the start-shard pipeline (--shard starts, --matches 1)")
        return False, "starts"
    if world == 1:
        return False, "matches"
    if shard != "starts" and strong != (shard in ("closure", "level")):  # start shards: either scaling
        raise ValueError(f"--shard {shard} does not belong to --scaling {scaling}")
    if shard != "matches" and matches != 1:
        raise ValueError("--matches > 1 runs with --shard matches (or N = 1)")
    return strong, shard


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); N > 1 without WORLD_SIZE set starts the N rank processes itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="metric", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="", choices=["", "strong", "weak"],
                    help="N>1: weak = per-GPU work fixed; strong = the workload's content split across ranks (one "
                         "match); default per workload (N_GT_1_DEFAULT: metric/config2 weak start shards, config4 "
                         "strong start shards on its 1,024 chars, config3/config5 strong closure shards)")
    ap.add_argument("--shard", default="", choices=["", "matches", "starts", "closure", "level"],
                    help="weak: starts (default; start-offset shards + RCCL all_gather + OR on rank 0) or matches "
                         "(independent matches per rank, no data-path collective); strong: closure (default; each "
                         "rank runs the dependency closure of its part of the top's inputs, one gather to rank 0) or "
                         "level (job slices per level, all-gathered level by level)")
    ap.add_argument("--one-rank-group", action="store_true",
                    help="N = 1: run the N > 1 start-shard pipeline (process group, stream-ordered export, "
                         "all_gather, OR on rank 0) with a one-rank group of --dist-backend, so the collective "
                         "path runs on a one-GPU box")
    ap.add_argument("--spawn-probe", action="store_true",
                    help="launcher test: the ranks meet over gloo and rank 0 prints who ran (no GPU)")
    ap.add_argument("--weak-matches-steps", type=int, default=-1,
                    help="--shard starts: steps of the secondary weak-by-matches timing (-1: --steps; 0: skip)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="N=1: secondary record of C matches in flight on C contexts (streams) of the GPU, "
                         "dealt round-robin (0: skip)")
    ap.add_argument("--lanes", type=int, default=4,
                    help="N=1: secondary record of matches in flight on the lanes (streams) of ONE context with one "
                         "key (fr_set_lanes; 0: skip)")
    ap.add_argument("--start-parts", type=int, default=0, choices=range(0, 17), metavar="{0..16}",
                    help="start shards: booleans per rank per match (fr_has_match_parts); 0: 16 // world (1 = "
                         "one boolean per rank, an extra OR level)")
    ap.add_argument("--faithful-steps", type=int, default=1,
                    help="N=1 metric: timed matches of the reference-structured lowering (FR_LOWER_FAITHFUL) "
                         "for the `faithful` sub-record (0: skip)")
    ap.add_argument("--matches", type=int, default=1, help="matches per rank per step (fr_has_match_batch)")
    ap.add_argument("--chars", type=int, default=0, help="content chars (strong: total; weak: per GPU); 0: workload's")
    ap.add_argument("--pattern", default="", help="override the workload's pattern")
    ap.add_argument("--content", default="", choices=["", "printable", "alnum", "letters", "config5"])
    ap.add_argument("--params", default="k1n2048", choices=["k1n2048", "k2n1024"])
    ap.add_argument("--ring", default="auto", choices=["auto", "fft", "rns"])
    ap.add_argument("--engine", default="auto", choices=["auto", "enumerate", "merged"])
    ap.add_argument("--lowering", default="threshold", choices=["threshold", "faithful", "faithful_tree"])
    ap.add_argument("--cpu-sample", type=int, default=2048,
                    help="gates in the CPU baseline sample (0: skip; 2048 ~ 10 s on 16 threads)")
    ap.add_argument("--cpu-match-max-jobs", type=int, default=2000, help="largest schedule the CPU match runs")
    ap.add_argument("--saturate", type=int, default=2048, help="gates in the saturated throughput probe (0: skip)")
    ap.add_argument("--no-power", action="store_true", help="no energy-accumulator readings (amdsmi) around the timed regions")
    ap.add_argument("--saturate-iters", type=int, default=10,
                    help="back-to-back launches the saturated probe times (after one warm-up launch)")
    ap.add_argument("--fresh-steps", type=int, default=5,
                    help="N=1: matches on newly encrypted content (encryption outside the timing; 0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 collectives (nccl = RCCL over xGMI; gloo only to rehearse ranks sharing one GPU)")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds a rendezvous or collective may wait before the rank aborts with an error "
                         "(init_process_group timeout; RCCL async error handling tears the rank down)")
    ap.add_argument("--job-timeout", type=float, default=1500.0,
                    help="--gpus N without a launcher: seconds before the spawned ranks are killed (0: none)")
    ap.add_argument("--strong-starts-steps", type=int, default=-1,
                    help="N>1: steps of the secondary `strong_starts` record (the workload's named length split by "
                         "start offsets; -1: --steps; 0: skip)")
    ap.add_argument("--faithful-tree-steps", type=int, default=3,
                    help="N=1 metric: timed matches of the reference op mix with its AND/OR chains rebalanced "
                         "(FR_LOWER_FAITHFUL_TREE) for the `faithful_tree` sub-record (0: skip)")
    ap.add_argument("--probe", default="1,16,254",
                    help="comma-separated batch sizes: blind-rotation ms per launch vs batch ('' to skip)")
    ap.add_argument("--out", default="", help="also write the JSON line to this file (rank 0)")
    ap.add_argument("--pmc", default="",
                    help="PMC summary of the BR kernel (tools/pmc_summary.py); default: the newest profiles/r0N/"
                         "pmc_summary.json at k1n2048, pmc_summary_k2n1024.json at k2n1024")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], args.job_timeout))
    if env_world is not None and int(env_world) != args.gpus:
        ap.error(f"--gpus {args.gpus} disagrees with WORLD_SIZE={env_world} from the launcher")
    if args.spawn_probe:
        spawn_probe(int(env_world or 1), int(os.environ.get("RANK", "0")))
        return
    if not args.pmc:  # the newest round's PMC summary of this parameter point
        name = "pmc_summary.json" if args.params == "k1n2048" else f"pmc_summary_{args.params}.json"
        cands = [os.path.join(REPO, "profiles", r, name) for r in ("r06", "r05", "r04", "r03")]
        args.pmc = next((c for c in cands if os.path.exists(c)), cands[-1])
    if args.matches < 1:
        ap.error("--matches must be >= 1")

    W = WORKLOADS[args.workload]
    pattern = args.pattern or W["pattern"]
    kind = args.content or W["content"]
    grammar = W.get("grammar", F.GRAMMAR_REFERENCE)
    engine = {"auto": F.ENGINE_AUTO, "enumerate": F.ENGINE_ENUMERATE, "merged": F.ENGINE_MERGED}[args.engine]
    lowering = {"threshold": F.LOWER_THRESHOLD, "faithful": F.LOWER_FAITHFUL,
                "faithful_tree": F.LOWER_FAITHFUL_TREE}[args.lowering]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1:
        args.scaling, args.shard = default_mode(args.workload, args.scaling, args.shard)
    try:
        strong, shard = resolve_mode(args.scaling, args.shard, world, args.matches, args.one_rank_group)
    except ValueError as e:
        ap.error(str(e))
    import torch

    dist = None
    if world > 1 or args.one_rank_group:
        # counting devices does not initialise the GPU on this image
        msg = nccl_device_guard(args.dist_backend, local_world, torch.cuda.device_count())
        if msg:
            ap.error(msg)
    # one process per GPU; only a gloo rehearsal (ranks beyond the visible devices on a
    # one-GPU box) shares devices round-robin
    device = local_rank % max(1, torch.cuda.device_count())
    if world > 1 or args.one_rank_group:
        import datetime

        import torch.distributed as dist

        if world == 1:  # a one-rank group without a launcher
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # a collective stuck past --dist-timeout aborts the rank (RCCL watchdog) instead of hanging the node
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        torch.cuda.set_device(device)
        dist.init_process_group(args.dist_backend, timeout=datetime.timedelta(seconds=args.dist_timeout))
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
    M = args.matches
    starts = shard == "starts"
    L = chars * world if starts and not strong else chars  # weak start shards: --chars per GPU

    def plant(m):
        """content of match m of this rank (weak matches: every rank its own)"""
        return make_content(kind, L, seed=(rank * M + m if shard == "matches" else 0))

    contents = [plant(m) for m in range(M)]
    content = contents[0]
    expected = [F.plain_match(c, pattern, engine=engine, grammar=grammar, lowering=lowering).result_lowered
                for c in contents]
    # content each rank holds: the window its starts read (start shards), else all of it
    if starts:
        lo, hi = F.shard_starts(L, world, rank)
        wlo, whi = F.content_window(L, pattern, lo, hi, lowering=lowering, engine=engine, grammar=grammar)
    else:
        lo, hi, wlo, whi = 0, L, 0, L

    lwes0 = []  # the first content's LWEs (the CPU baseline evaluates the same words)

    def encrypt(c, seed, keep=False):
        hs = [F.NULL_CT] * L
        if whi > wlo:
            msgs = [(ch >> (2 * b)) & 3 for ch in c[wlo:whi] for b in range(4)]
            blocks = ctx.encrypt_blocks(msgs, seed=seed, first_block=4 * wlo).reshape(whi - wlo, 4, ctx.lwe_len)
            if keep:
                lwes0.append(blocks)
            for i, h in enumerate(ctx.upload_radix(blocks)):
                hs[wlo + i] = h
        return hs

    batch = [encrypt(c, 7 + 1000 * rank + m, keep=m == 0) for m, c in enumerate(contents)]
    handles = batch[0]
    handles_np = np.asarray(handles, dtype=np.uint32)  # passed without a per-call ctypes copy

    plan = None
    phase = {}
    gather = F.torch_all_gather() if dist is not None else None
    if strong and not starts:
        plan = F.ShardPlan(ctx, handles, pattern)
        sched = F.schedule_match(L, pattern, lowering=lowering, engine=engine, grammar=grammar)
        if shard == "closure":
            cparts = F.closure_parts(sched, world)  # once: the host derivation costs ms per call
            runs, _, top = cparts
            closure_rot = [sum(b - a for rl in runs[r] for a, b in rl) for r in range(world)]
            closure_rot[0] += sum(b - a for rl in top for a, b in rl)

    def step(times=None):
        """one step; returns ([result handles] on rank 0 (else []), rotations run by this rank, stats)"""
        if shard == "matches":
            if M == 1:
                out, st = ctx.has_match(handles_np, pattern)
                return [out], st.blind_rotations, st
            outs, st = ctx.has_match_batch(batch, pattern)
            return outs, st.blind_rotations, st
        if shard == "closure":
            F.run_closure_sharded(plan, sched, world, rank, gather, cparts, times=times)
            if rank == 0:  # the match's rotations (jobs two ranks both ran count once)
                t = time.perf_counter()
                out, st = plan.finish()
                if times is not None:
                    times["top_ms"] = times.get("top_ms", 0.0) + (time.perf_counter() - t) * 1e3
                return [out], len(sched.jobs), st
            return [], 0, plan.stats
        if shard == "level":
            F.run_sharded(plan, world, rank, gather, times=times)
            mine = sum(len(range(*F.job_slice(plan.jobs(l), world, rank))) for l in range(plan.levels - 1))
            if rank == 0:
                t = time.perf_counter()
                out, st = plan.finish()
                if times is not None:
                    times["top_ms"] = times.get("top_ms", 0.0) + (time.perf_counter() - t) * 1e3
                return [out], mine + plan.jobs(plan.levels - 1), st
            return [], mine, plan.stats
        raise AssertionError("start shards run starts_pipeline")

    rccl = args.dist_backend == "nccl"
    coll_name = "RCCL" if rccl else "gloo (host-staged)"
    lib_stream = (torch.cuda.ExternalStream(ctx.stream_ptr(), device=torch.device("cuda", device))
                  if starts or dist is not None else None)

    def starts_job(Lj, seed):
        """this rank's part of a start-sharded match over Lj chars of the workload's content:
        its start range, the content window those starts read (encrypted into this rank's
        arena, nothing else), the expected bit"""
        cj = make_content(kind, Lj, seed=0)
        jlo, jhi = F.shard_starts(Lj, world, rank)
        jwlo, jwhi = F.content_window(Lj, pattern, jlo, jhi, lowering=lowering, engine=engine, grammar=grammar)
        hs = [F.NULL_CT] * Lj
        if jwhi > jwlo:
            msgs = [(ch >> (2 * b)) & 3 for ch in cj[jwlo:jwhi] for b in range(4)]
            blocks = ctx.encrypt_blocks(msgs, seed=seed, first_block=4 * jwlo).reshape(jwhi - jwlo, 4, ctx.lwe_len)
            for i, h in enumerate(ctx.upload_radix(blocks)):
                hs[jwlo + i] = h
        exp = F.plain_match(cj, pattern, engine=engine, grammar=grammar, lowering=lowering).result_lowered
        return {"handles": np.asarray(hs, dtype=np.uint32), "lo": jlo, "hi": jhi, "L": Lj, "expected": exp,
                "window": (jwlo, jwhi)}

    # parts per rank (fr_has_match_parts): each rank's OR tree stops at <= P booleans, so the
    # world * P gathered booleans are ONE threshold OR: the tree's last level runs once, on
    # rank 0, instead of once per rank plus once to combine (/abc/ on 256 chars at N = 2..8:
    # 4 levels, as at N = 1, instead of 5)
    P = args.start_parts or (max(1, 16 // world) if world <= 16 else 1)

    def starts_pipeline(n, times=None, job=None):
        """n start-sharded matches (north_star's per-start-offset variants + final bitor,
        engine.rs:15-35): per step every rank enqueues its start range's match as <= P
        parts, exports them device to device into that step's row (stream-ordered) and all-gathers the
        row (RCCL on torch's stream, ordered after the export by an event on the library's
        stream; the host never waits between matches).  Rank 0 then ORs every step's
        gathered booleans in ONE launch (n independent threshold ORs).  gloo (a rehearsal:
        ranks sharing one GPU) stages the gather through the host.  job: starts_job(...)
        (default: the timed workload's).  Returns ([result per step] on rank 0, rotations
        this rank ran, last stats)."""
        jh, jlo, jhi = (handles_np, lo, hi) if job is None else (job["handles"], job["lo"], job["hi"])
        # every row is overwritten by an export on the library's stream, which must not
        # overtake the allocation's work on torch's stream
        send = torch.empty((n, P, ctx.lwe_len), dtype=torch.int64, device=f"cuda:{device}")
        recv = torch.empty((n, world, P, ctx.lwe_len), dtype=torch.int64, device=f"cuda:{device}")
        lib_stream.wait_stream(torch.cuda.current_stream())
        rot, st = 0, None
        for i in range(n):
            t = time.perf_counter()
            if P > 1:  # up to P parts; a short list repeats its first (OR is idempotent)
                outs_i, st = ctx.has_match_parts(jh, pattern, jlo, jhi, P)
                outs_i += [outs_i[0]] * (P - len(outs_i))
            else:
                out, st = ctx.has_match(jh, pattern, jlo, jhi)
                outs_i = [out]
            rot += st.blind_rotations
            if rccl:
                ctx.export_bool_device_async(outs_i, send[i].data_ptr())
                ev = torch.cuda.Event()
                ev.record(lib_stream)
                torch.cuda.current_stream().wait_event(ev)
            else:
                ctx.export_bool_device(outs_i, send[i].data_ptr())
            for h in set(outs_i):
                ctx.release(h)  # stream-ordered: a later user of its slot runs after the export
            t2 = time.perf_counter()
            if rccl:
                dist.all_gather_into_tensor(recv[i].view(-1), send[i].view(-1))
            else:
                for r, b in enumerate(gather(send[i].view(-1))):
                    recv[i, r].copy_(b.view(P, -1))
            if times is not None:
                times["starts_ms"] = times.get("starts_ms", 0.0) + (t2 - t) * 1e3
                times["gather_ms"] = times.get("gather_ms", 0.0) + (time.perf_counter() - t2) * 1e3
        torch.cuda.synchronize()  # the gathers (torch's stream) before the library reads recv
        if rank != 0:
            return [], rot, st
        t = time.perf_counter()
        parts = ctx.import_bool_device(recv.data_ptr(), n * world * P)
        g = world * P  # booleans per step
        if g <= 16:
            res = ctx.or_each([parts[i * g:(i + 1) * g] for i in range(n)])
            rot += n
        else:
            res = [ctx.or_many(parts[i * g:(i + 1) * g]) for i in range(n)]
            rot += 2 * n
        for h in parts:
            ctx.release(h)
        if times is not None:
            times["or_ms"] = times.get("or_ms", 0.0) + (time.perf_counter() - t) * 1e3
        return res, rot, st

    first_call = None
    for _ in range(args.warmup):
        t = time.perf_counter()
        o, _, st0 = starts_pipeline(1) if starts else step()
        if first_call is None:  # cold call: parse, record, lower, compile, plan upload, and its device time
            torch.cuda.synchronize()
            first_call = {"host_ms": st0.host_ms, "wall_ms": (time.perf_counter() - t) * 1e3,
                          "plan_cached": st0.plan_cached}
        for h in o:
            ctx.release(h)

    meter = EnergyMeter(torch.cuda.get_device_properties(device)) if rank == 0 and not args.no_power else None
    ctx.set_profiling(True)
    t_before = ctx.device_timers()
    barrier()
    e_timed0 = meter.read() if meter else None
    t0 = time.perf_counter()
    rot_local = 0
    host_ms = 0.0
    outs = []
    st = None
    if starts:
        step_outs, rot_local, st = starts_pipeline(args.steps, phase)
        outs = step_outs[-1:]
    for i in range(0 if starts else args.steps):
        o, rot, st = step(phase)
        rot_local += rot
        host_ms += st.host_ms if shard == "matches" else 0.0
        if i + 1 < args.steps:
            for h in o:
                ctx.release(h)
        else:
            outs = o
    barrier()
    elapsed = time.perf_counter() - t0
    e_timed1 = meter.read() if meter else None
    t_after = ctx.device_timers()
    ctx.set_profiling(False)
    ms_per_step_local = elapsed / args.steps * 1e3
    rotations_per_match_local = rot_local / args.steps / M

    per_rank = None
    if dist is not None:
        tt = torch.tensor([elapsed, float(rot_local)], dtype=torch.float64, device=coll_dev)
        mx = tt.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        elapsed, total_rot = float(mx[0]), float(tt[1])
        # per-rank diagnosis: wall ms per phase per step, rotations run
        keys = ["closure_ms", "gather_ms", "top_ms", "slices_ms", "import_ms", "starts_ms", "or_ms"]
        mine = torch.tensor([phase.get(kk, 0.0) / args.steps for kk in keys] +
                            [float(rot_local) / args.steps, elapsed * 1e3 / args.steps],
                            dtype=torch.float64, device=coll_dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = []
        for r, v in enumerate(allr):
            v = v.cpu().tolist()
            d = {"rank": r, "rotations_run": v[len(keys)], "step_ms": v[len(keys) + 1]}
            if shard == "closure":  # counted once toward value (rank 0) vs run on this rank (its closure)
                d["rotations_counted"], d["rotations_run"] = v[len(keys)], float(closure_rot[r])
            d.update({kk: round(x, 4) for kk, x in zip(keys, v) if kk in phase or x})
            per_rank.append(d)
    else:
        total_rot = float(rot_local)

    result = None
    words0 = None
    starts_ok = None
    if rank == 0:
        words = [ctx.download_radix(o) for o in outs]
        words0 = words[0][0] if words else None
        result = [ctx.decrypt_radix(w) for w in words]
        if starts:  # every step's OR, not just the last
            starts_ok = all(ctx.decrypt_radix(ctx.download_radix(o)) == expected[0] for o in step_outs)
            for o in step_outs:
                ctx.release(o)
            outs = []
        exp = expected if shard == "matches" else expected[:1]
        if result != exp:
            print(f"WARNING: decrypted results {result} != expected {exp}", file=sys.stderr)

    fresh = None
    if args.fresh_steps and world == 1 and M == 1:
        # newly encrypted content for every match (device encryption before the timing): the
        # template plan is replayed with each content's slots bound; timed like the replay
        # (back-to-back matches, one synchronise at the end)
        cs = [make_content(kind, L, seed=100 + i) for i in range(args.fresh_steps)]
        hss = [np.asarray(ctx.encrypt_upload_str(c, seed=500 + i), dtype=np.uint32) for i, c in enumerate(cs)]
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = [ctx.has_match(h, pattern) for h in hss]
        torch.cuda.synchronize()
        fresh_ms = (time.perf_counter() - t) * 1e3 / args.fresh_steps
        ok = all(ctx.decrypt_radix(ctx.download_radix(o)) ==
                 F.plain_match(c, pattern, engine=engine, grammar=grammar, lowering=lowering).result_lowered
                 for (o, _), c in zip(res, cs))
        fresh = {"fresh_content_ms": fresh_ms, "matches": args.fresh_steps,
                 "plan_cached": [int(stf.plan_cached) for _, stf in res], "results_ok": bool(ok),
                 "replay_ms": elapsed / args.steps * 1e3}
        for (o, _), hs in zip(res, hss):
            for h in list(hs) + [o]:
                ctx.release(int(h))

    weak_matches = None
    wm_steps = args.steps if args.weak_matches_steps < 0 else args.weak_matches_steps
    if shard == "starts" and dist is not None and wm_steps > 0:
        # secondary record: weak scaling by matches (every rank one full-length match of
        # the workload on its own content per step, no data-path collective)
        own = make_content(kind, chars, seed=rank)
        own_hs = np.asarray(ctx.encrypt_upload_str(own, seed=9000 + rank), dtype=np.uint32)
        o, _ = ctx.has_match(own_hs, pattern)  # warm-up (plan)
        ctx.release(o)
        barrier()
        t = time.perf_counter()
        wrot = 0
        for i in range(wm_steps):
            o, stw = ctx.has_match(own_hs, pattern)
            wrot += stw.blind_rotations
            if i + 1 < wm_steps:
                ctx.release(o)
        barrier()
        wel = time.perf_counter() - t
        ok = ctx.decrypt_radix(ctx.download_radix(o)) == F.plain_match(
            own, pattern, engine=engine, grammar=grammar, lowering=lowering).result_lowered
        ctx.release(o)
        tt = torch.tensor([wel, float(wrot), float(ok)], dtype=torch.float64, device=coll_dev)
        mx, sm = tt[:1].clone(), tt[1:].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        weak_matches = {"value": float(sm[0]) / float(mx[0]), "unit": "gate-bootstraps/s",
                        "ms_per_step": float(mx[0]) * 1e3 / wm_steps, "steps": wm_steps,
                        "workload": f"{pattern} on {chars} chars, one match per rank per step on its own content",
                        "results_ok_ranks": int(sm[1]), "note": "secondary: weak scaling by matches, never `value`"}
        for h in own_hs:
            ctx.release(int(h))

    strong_starts = None
    ss_steps = args.steps if args.strong_starts_steps < 0 else args.strong_starts_steps
    if starts and strong and dist is not None:
        strong_starts = {"same_as_value": True,
                         "note": "the timed region is already the named length split by start offsets"}
    elif dist is not None and ss_steps > 0:
        # secondary record: the workload's NAMED length (256 chars for the metric, 1,024 for
        # config 4, ...) split by start offsets across the ranks -- north_star's split at
        # BASELINE's length, strong scaling -- beside a value on other terms; never `value`
        job = starts_job(chars, 7 + 1000 * rank + 77)
        for h in starts_pipeline(1, job=job)[0]:  # warm-up (plan)
            ctx.release(h)
        sphase = {}
        barrier()
        t = time.perf_counter()
        s_outs, s_rot, _ = starts_pipeline(ss_steps, sphase, job=job)
        barrier()
        sel = time.perf_counter() - t
        s_ok = all(ctx.decrypt_radix(ctx.download_radix(o)) == job["expected"] for o in s_outs) if rank == 0 else True
        for o in s_outs:
            ctx.release(o)
        tt = torch.tensor([sel, float(s_rot), float(s_ok)], dtype=torch.float64, device=coll_dev)
        mx, sm = tt[:1].clone(), tt[1:].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        skeys = ["starts_ms", "gather_ms", "or_ms"]
        mine = torch.tensor([sphase.get(kk, 0.0) / ss_steps for kk in skeys] + [float(s_rot) / ss_steps, sel * 1e3 / ss_steps],
                            dtype=torch.float64, device=coll_dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        s_per_rank = []
        for r, v in enumerate(allr):
            v = v.cpu().tolist()
            d = {"rank": r, "rotations_run": v[len(skeys)], "step_ms": v[len(skeys) + 1]}
            d.update({kk: round(x, 4) for kk, x in zip(skeys, v) if x})
            s_per_rank.append(d)
        strong_starts = {"value": float(sm[0]) / float(mx[0]), "unit": "gate-bootstraps/s",
                         "ms_per_step": float(mx[0]) * 1e3 / ss_steps, "steps": ss_steps,
                         "content_chars": job["L"], "scaling": "strong", "parts_per_rank": P,
                         "workload": f"{pattern} on {job['L']} chars (the workload's named length) split by start "
                                     f"offsets over {world} ranks, {coll_name} gather, OR on rank 0",
                         "results_ok_steps": bool(sm[1] >= world), "result_expected": job["expected"],
                         "per_rank": s_per_rank, "note": "secondary: never `value`"}
        for h in job["handles"]:
            if h != F.NULL_CT:
                ctx.release(int(h))

    inflight = None
    if args.inflight > 1 and world == 1 and M == 1 and rank == 0 and not starts:
        # serving view: C independent single matches in flight, one per context (each context
        # its own stream, arena and copy of the keys), dealt round-robin; each match is the
        # full workload match, bit-identical to the timed region's
        ictx, ihs = [ctx], [handles_np]
        for i in range(1, args.inflight):
            c = F.Context(device, params)
            c.load_client_key(blob)
            c.gen_server_key(SERVER_KEY_SEED)
            c.set_lowering(lowering)
            c.set_engine(engine)
            c.set_grammar(grammar)
            ictx.append(c)
            ihs.append(np.asarray(c.upload_radix(lwes0[0] if lwes0 else c.encrypt_str(content, seed=7)),
                                  dtype=np.uint32))
        for c, h in zip(ictx, ihs):  # plans
            c.release(c.has_match(h, pattern)[0])
        torch.cuda.synchronize()
        nm = max(args.steps, 2 * args.inflight)
        t = time.perf_counter()
        outs_if = [(i % args.inflight, ictx[i % args.inflight].has_match(ihs[i % args.inflight], pattern)[0])
                   for i in range(nm)]
        torch.cuda.synchronize()
        ims = (time.perf_counter() - t) * 1e3 / nm
        w_if = [ictx[k].download_radix(o) for k, o in outs_if]
        same = all(np.array_equal(w[0], words0) for w in w_if) if words0 is not None else None
        for k, o in outs_if:
            ictx[k].release(o)
        inflight = {"contexts": args.inflight, "matches": nm, "ms_per_match_amortised": ims,
                    "value": rotations_per_match_local / (ims / 1e3), "unit": "gate-bootstraps/s",
                    "bit_identical_to_timed_region": same,
                    "note": "secondary, serving view: independent single matches in flight on separate contexts "
                            "(streams); each match's own latency stays match_ms. Never `value`."}
        for c in ictx[1:]:
            c.close()

    inflight_1ctx = None
    if args.lanes > 1 and world == 1 and M == 1 and rank == 0 and not starts:
        # serving with ONE key: the same matches in flight on the lanes (streams) of this
        # context (fr_set_lanes), each lane its own plan copy; consecutive asynchronous
        # matches round-robin over the lanes, so a match's small levels share the chip with
        # the next match's first level
        ctx.set_lanes(args.lanes)
        try:
            for _ in range(args.lanes):  # each lane's plan
                ctx.release(ctx.has_match(handles_np, pattern)[0])
            torch.cuda.synchronize()
            ctx.download_radix(handles[next(i for i, h in enumerate(handles) if h != F.NULL_CT)])
            nm = max(args.steps, 4 * args.lanes)
            t = time.perf_counter()
            outs_l = [ctx.has_match(handles_np, pattern)[0] for _ in range(nm)]
            w_l = ctx.download_radix(outs_l[-1])  # synchronises every lane
            lms = (time.perf_counter() - t) * 1e3 / nm
            same = all(np.array_equal(ctx.download_radix(o)[0], words0) for o in outs_l) if words0 is not None else None
            for o in outs_l:
                ctx.release(o)
        finally:
            ctx.set_lanes(1)
        inflight_1ctx = {"lanes": args.lanes, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "matches": nm, "ms_per_match_amortised": lms,
                         "value": rotations_per_match_local / (lms / 1e3), "unit": "gate-bootstraps/s",
                         "bit_identical_to_timed_region": same, "result_decrypted": ctx.decrypt_radix(w_l),
                         "note": "secondary, serving view with one key: matches in flight on the lanes (streams) of "
                                 "one context (fr_set_lanes), each lane its own plan copy. Never `value`."}

    step_latency = None
    if starts:
        # latency of one start-sharded match end to end (match, export, gather, the OR on
        # rank 0), synchronised before and after; the timed region pipelines these
        lat_ms = []
        for _ in range(3):
            barrier()
            t = time.perf_counter()
            o, _, _ = starts_pipeline(1)
            barrier()
            lat_ms.append((time.perf_counter() - t) * 1e3)
            for h in o:
                ctx.release(h)
        step_latency = {"ms_min": min(lat_ms), "ms_mean": sum(lat_ms) / len(lat_ms), "runs": len(lat_ms),
                        "what": "one start-sharded match end to end (rank 0's view after barriers): the ranks' "
                                "matches, the boolean all-gather and the OR on rank 0"}

    def lowering_record(mode, steps, label):
        """the same content's match under another lowering (one gate group per smart_* op,
        execution.rs:64-195): its PBS count and levels are the reference's op structure"""
        ctx.set_lowering(mode)
        t = time.perf_counter()
        o, stf = ctx.has_match(handles_np, pattern)
        torch.cuda.synchronize()
        cold_ms = (time.perf_counter() - t) * 1e3
        ctx.release(o)
        t = time.perf_counter()
        for i in range(steps):
            o, stf = ctx.has_match(handles_np, pattern)
            if i + 1 < steps:
                ctx.release(o)
        torch.cuda.synchronize()
        fms = (time.perf_counter() - t) * 1e3 / steps
        fres = ctx.decrypt_radix(ctx.download_radix(o))
        ctx.release(o)
        ctx.set_lowering(lowering)
        return {"lowering": label, "match_ms": fms, "first_call_ms": cold_ms, "steps": steps,
                "pbs": int(stf.pbs), "blind_rotations": int(stf.blind_rotations), "levels": int(stf.levels),
                "pbs_per_s": stf.pbs / (fms / 1e3), "result_decrypted": fres, "result_expected": expected[0],
                "vs_threshold_ms": ms_per_step_local}

    faithful = faithful_tree = None
    if world == 1 and M == 1 and rank == 0 and lowering == F.LOWER_THRESHOLD and not starts:
        if args.faithful_steps > 0:
            faithful = lowering_record(F.LOWER_FAITHFUL, args.faithful_steps,
                                       "faithful (FR_LOWER_FAITHFUL: eq/gt/le = 3 PBS, and/or = 1, not linear; the "
                                       "reference's serial fold, engine.rs:22-35)")
        if args.faithful_tree_steps > 0:
            # the reference's op mix (the same gates as `faithful`) with its AND/OR chains
            # rebalanced into binary trees of least depth: log depth
            faithful_tree = lowering_record(F.LOWER_FAITHFUL_TREE, args.faithful_tree_steps,
                                            "faithful_tree (FR_LOWER_FAITHFUL_TREE: the faithful gates, eq/gt/le = 3 "
                                            "PBS, and/or = 1, with every unshared AND/OR chain rebalanced; never "
                                            "`value`)")

    kernel = None
    e_sat0 = e_sat1 = None
    if args.saturate and rank == 0:
        src = [h for h in handles if h != F.NULL_CT]
        hs = [src[i % len(src)] for i in range(args.saturate)]
        ctx.dev_bench_pbs(hs, 1)  # warm-up, as the latency probe below
        it = max(1, args.saturate_iters)
        e_sat0 = meter.read() if meter else None
        br_sat, tot_sat = ctx.dev_bench_pbs(hs, it)
        e_sat1 = meter.read() if meter else None
        kernel = {"gates_per_launch": args.saturate, "launches": it, "br_ms_per_launch": br_sat / it,
                  "pbs_per_s": it * args.saturate / (tot_sat / 1e3),
                  "br_pbs_per_s": it * args.saturate / (br_sat / 1e3)}

    probe = None
    if args.probe.strip("' ") and rank == 0:
        src = [h for h in handles if h != F.NULL_CT]
        probe = {}
        for cnt in [int(x) for x in args.probe.replace("'", "").split(",") if x.strip("' ")]:
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
    fpp = algorithmic_flops_per_pbs(params)
    br_ms = t_after["br_ms"] - t_before["br_ms"]
    br_launches = t_after["br_launches"] - t_before["br_launches"]
    br_gates = t_after["br_gates"] - t_before["br_gates"]
    lat = {kk: t_after[kk] - t_before[kk] for kk in ("lat_br_ms", "lat_launches", "lat_gates",
                                                     "pair_br_ms", "pair_launches", "pair_gates")}
    cus = 256

    def shape_line(name, ms, launches, gates, per_wg=1):
        """one launch shape: algorithmic TFLOP/s, also per active CU (min(workgroups, 256) CUs; per_wg
        bootstraps per workgroup); the contract's HBM figures at this shape: algorithmic GGSW bytes
        (bpp per bootstrap) and the PMC's physical bytes per launch of the shape, over its launch time"""
        if ms <= 0 or launches == 0:
            return None
        tf = gates * fpp / (ms / 1e3) / 1e12
        active = min(gates / launches / per_wg, cus)
        avg_s = ms / launches / 1e3
        alg = gates / launches * bpp / avg_s / 1e9
        phys_b = (pmc or {}).get("traffic_per_shape", {}).get(name)
        phys = phys_b / avg_s / 1e9 if phys_b else None
        return {"launches": int(launches), "bootstraps_per_launch": gates / launches, "avg_ms": ms / launches,
                "achieved_tflops": tf, "frac": tf / FP64_VECTOR_PEAK_TFLOPS,
                "frac_of_active_cus": tf / (FP64_VECTOR_PEAK_TFLOPS * active / cus),
                "hbm_algorithmic_GBps": alg, "hbm_algorithmic_frac": alg / HBM_PEAK_GBS,
                "hbm_physical_bytes_per_launch": phys_b, "hbm_physical_GBps": phys,
                "hbm_physical_frac": phys / HBM_PEAK_GBS if phys is not None else None}

    pmc = pmc_figures(params, args.pmc)
    per_shape = {
        "latency": shape_line("latency", lat["lat_br_ms"], lat["lat_launches"], lat["lat_gates"]),
        "pair": shape_line("pair", lat["pair_br_ms"], lat["pair_launches"], lat["pair_gates"], 2),
        "throughput": shape_line("throughput", br_ms - lat["lat_br_ms"] - lat["pair_br_ms"],
                                 br_launches - lat["lat_launches"] - lat["pair_launches"],
                                 br_gates - lat["lat_gates"] - lat["pair_gates"]),
    }
    achieved_tf = br_gates * fpp / (br_ms / 1e3) / 1e12 if br_ms > 0 else 0.0
    alg_gbs = (br_gates * bpp) / (br_ms / 1e3) / 1e9 if br_ms > 0 else 0.0
    br_avg_ms = br_ms / max(br_launches, 1)
    phys = pmc["traffic"] / (br_avg_ms / 1e3) / 1e9 if pmc and pmc.get("traffic") and br_avg_ms > 0 else None
    cpu = None
    if args.cpu_sample > 0 and world == 1 and dist is None:  # its word check reads the plain match's output
        cpu = cpu_baseline(params, content, pattern, grammar, engine, lowering, args.cpu_sample,
                           args.cpu_match_max_jobs, lwes0[0] if lwes0 else None, words0)
    ms_per_step = elapsed / args.steps * 1e3
    ring_name = "fft" if params.ring == F.RING_FFT else "rns"
    coll = "RCCL" if args.dist_backend == "nccl" else "gloo (host-staged)"
    if world == 1 and not starts:
        par = "single GPU" + (f", {M} matches per step in shared launches" if M > 1 else "")
    elif shard == "matches":
        par = (f"dp{world}: {M} independent match(es) per rank per step on its own content, no data-path collective "
               f"(max-over-ranks timing)")
    elif shard == "closure":
        par = (f"closure-sharded x{world} (each rank runs the dependency closure of its part of the top's inputs, "
               f"one {coll} all_gather of those LWEs, rank 0 runs the top)")
    elif shard == "level":
        par = f"level-sharded x{world} (job slices per level, {coll} all_gather of each level's LWEs)"
    else:
        par = (f"start-offset shards x{world} (each rank its start range on its content window; {coll} "
               f"all_gather of the per-rank booleans, stream-ordered after each match; rank 0 ORs every step's "
               f"booleans in one launch at the end of the timed region)")
    work = f"{args.workload}: {pattern} on {L} chars" + (f" ({chars} per GPU)" if starts and not strong else "")
    if M > 1 or (world > 1 and shard == "matches"):
        work += f", {M} match(es) per GPU per step"
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
        "dtype_note": "LWE/GLWE words are u64 on the 2^64 torus; the blind rotation computes in f64 "
                      "(negacyclic FFT products and an f64 accumulator, tfhe-rs's own arithmetic class, "
                      "Cargo.lock:110-114 concrete-fft); keyswitch in exact int8 MFMA limbs",
        "data": "synthetic: seeded content, real encryptions under the reference fixture client key",
        "config": {"workload": work, "content_chars": L, "matches_per_gpu": M, "params": args.params,
                   "ring": ring_name, "lowering": args.lowering, "engine": args.engine, "content": kind,
                   "scaling": "strong" if strong else "weak", "shard": shard, "parallelism": par,
                   "start_parts": P if starts else None},
        "match_ms": ms_per_step,
        "blind_rotations_per_step": total_rot / args.steps,
        "lut_outputs_per_match": float(st.pbs) / (M if shard == "matches" else 1),
        "levels": st.levels,
        "host_ms_per_step": host_ms / args.steps if shard == "matches" else None,
        "rotations_run_per_rank": closure_rot if shard == "closure" else None,
        "per_rank": per_rank,
        "first_call": first_call,
        "fresh_content": fresh,
        "result_decrypted": result,
        "result_expected": expected if shard == "matches" else expected[:1],
        "keygen_s": t_key,
        "roofline": {
            "bound": "valu",
            "achieved": achieved_tf,
            "peak": FP64_VECTOR_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / FP64_VECTOR_PEAK_TFLOPS,
            "traffic": pmc["traffic"] if pmc else None,
            "kernel": "k_blind_rotate_fft" if params.ring == F.RING_FFT else "k_blind_rotate",
            "achieved_is": "algorithmic f64 FLOP per bootstrap (ceil(n/2) steps x [2(k+1) FFTs at 5 M log2 M + "
                           "3 (k+1)^2 complex MACs per slot]) x bootstraps / BR kernel time (HIP events, timed "
                           "region); peak = FP64 vector spec",
            "flops_per_pbs": fpp,
            "br_launches": br_launches,
            "br_avg_ms": br_avg_ms,
            "br_gates_per_launch": br_gates / max(br_launches, 1),
            "per_shape": per_shape,
            "valu_issue": None if not pmc or pmc.get("valu_per_cu_clk") is None else {
                "achieved": pmc["valu_per_cu_clk"],
                "unit": "VALU wave64 instructions per active-CU clock (SQ_INSTS_VALU, rocprofv3 PMC)",
                "frac_spec": pmc["valu_per_cu_clk"] / VALU_SPEC_PER_CU_CLK,
                "frac_measured_peak": pmc["valu_per_cu_clk"] / VALU_F64_PEAK,
                "peaks": {"spec": VALU_SPEC_PER_CU_CLK, "measured_v_fma_f64": VALU_F64_PEAK},
            },
            "hbm": {
                "physical_GBps": phys,
                "physical_frac": phys / HBM_PEAK_GBS if phys is not None else None,
                "physical_is": "PMC HBM bytes per BR launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) / "
                               "average BR launch time",
                "algorithmic_GBps": alg_gbs,
                "algorithmic_is": f"n (k+1)^2 l N 8 = {bpp} B of GGSW per bootstrap x bootstraps / BR time: a "
                                  "normalisation, not a physical rate -- bootstraps in flight share each step's key "
                                  "through the XCD's L2, so at >= 512 bootstraps per launch it exceeds the 8 TB/s peak",
            },
            "north_star_hbm": north_star_hbm(per_shape),
            "pmc_source": pmc["source"] if pmc else None,
            "pmc_stale": pmc["stale"] if pmc else None,
        },
        "results_ok_steps": starts_ok,
        "step_latency": step_latency,
        "inflight": inflight,
        "inflight_1ctx": inflight_1ctx,
        "weak_matches": weak_matches,
        "faithful": faithful,
        "faithful_tree": faithful_tree,
        "strong_starts": strong_starts,
        # BASELINE's named length (256 chars for the metric) at this N, whatever `value`'s
        # sharding: the field a 1 -> 8 GPU scaling plot of the named workload reads
        "named_length": named_length_record(total_rot / elapsed, ms_per_step, L, W["chars"], M, world, strong,
                                            starts_ok if starts_ok is not None else
                                            (result == (expected if shard == "matches" else expected[:1])),
                                            strong_starts, args.steps),
        "kernel_saturated": kernel,
        # socket power and energy per bootstrap of rank 0's GPU (driver energy accumulator) over the
        # timed region and the saturated probe; the board's power cap bounds the saturated rate
        "power": None if meter is None or meter.h is None else {
            "source": "amdsmi energy accumulator (socket), read outside each region; rank 0's GPU",
            "cap_w": meter.cap_w,
            # ranks sharing one GPU (gloo rehearsals): the socket's energy is every rank's work
            "timed_region": meter.region(e_timed0, e_timed1,
                                         rot_local if world <= torch.cuda.device_count() else None),
            "saturated": meter.region(e_sat0, e_sat1, kernel["launches"] * kernel["gates_per_launch"]) if kernel else None,
        },
        "latency_probe": probe,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(json.dumps(line) + "\n")
    if plan is not None:
        plan.free()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
