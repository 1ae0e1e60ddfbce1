"""bench.py's launcher path on the CPU: `--gpus N` with no WORLD_SIZE starts the N
rank processes itself (torch.distributed.run as a child, before any GPU call), an
external launcher's WORLD_SIZE must agree with --gpus, and the N > 1 default is
north_star's start-offset shards."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
sys.path.insert(0, REPO)


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_spawns_ranks(n):
    res = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--spawn-probe"], capture_output=True, text=True,
                         timeout=240, env=_env())
    assert res.returncode == 0, res.stderr[-2000:]
    lines = res.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), res.stdout  # one JSON line, from rank 0, nothing else
    d = json.loads(lines[0])
    assert d["spawn_probe"] and d["n_gpus"] == n and d["ranks"] == list(range(n))
    assert len(set(d["pids"])) == n
    assert len(set(d["parent_pids"])) == 1  # siblings under one launcher child of bench.py


def test_single_gpu_runs_in_process():
    res = subprocess.run([sys.executable, BENCH, "--spawn-probe"], capture_output=True, text=True, timeout=120,
                         env=_env())
    assert res.returncode == 0, res.stderr[-2000:]
    d = json.loads(res.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["ranks"] == [0]
    assert d["parent_pids"] == [os.getpid()]  # no launcher in between


def test_world_size_must_match_gpus():
    res = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--spawn-probe"], capture_output=True, text=True,
                         timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert res.returncode == 2 and "disagrees with WORLD_SIZE=2" in res.stderr


def test_mode_defaults():
    import bench
    assert bench.resolve_mode("weak", "", 1, 1) == (False, "matches")
    assert bench.resolve_mode("weak", "", 8, 1) == (False, "starts")
    assert bench.resolve_mode("weak", "matches", 8, 4) == (False, "matches")
    assert bench.resolve_mode("strong", "", 8, 1) == (True, "closure")
    assert bench.resolve_mode("strong", "level", 2, 1) == (True, "level")
    assert bench.resolve_mode("strong", "starts", 4, 1) == (True, "starts")  # fixed content, starts split
    # --one-rank-group: the start-shard pipeline over a one-rank process group
    assert bench.resolve_mode("weak", "", 1, 1, True) == (False, "starts")
    with pytest.raises(ValueError):
        bench.resolve_mode("weak", "matches", 1, 1, True)
    with pytest.raises(ValueError):
        bench.resolve_mode("weak", "closure", 2, 1)
    with pytest.raises(ValueError):
        bench.resolve_mode("weak", "starts", 2, 4)


def test_n_gt_1_defaults_measure_named_lengths():
    """N > 1 defaults per workload: the metric's value is weak start shards
    (N x 256 chars, the named 256 split as the `strong_starts` record); config 4's value is
    its named 1,024 chars split by start offsets; the anchored configs split one match by
    closures.  Explicit flags win."""
    import bench
    assert bench.default_mode("metric", "", "") == ("weak", "starts")
    assert bench.default_mode("config4", "", "") == ("strong", "starts")
    assert bench.default_mode("config5", "", "") == ("strong", "closure")
    assert bench.default_mode("config3", "", "") == ("strong", "closure")
    assert bench.default_mode("config4", "weak", "") == ("weak", "")
    assert bench.default_mode("config4", "", "closure") == ("strong", "closure")
    assert bench.resolve_mode(*bench.default_mode("config4", "", ""), 8, 1) == (True, "starts")
    assert bench.resolve_mode(*bench.default_mode("config5", "", ""), 8, 1) == (True, "closure")
    assert bench.resolve_mode(*bench.default_mode("metric", "", ""), 8, 1) == (False, "starts")


def test_named_length_record():
    """named_length: the named workload at this N, whatever `value`'s
    sharding -- `value` itself for one match of the named length (N = 1, or a strong split),
    the hoisted strong_starts record when `value` is weak start shards (N x the chars)"""
    import bench
    r = bench.named_length_record(1e5, 7.0, 256, 256, 1, 1, False, True, None, 20)
    assert r == {"chars": 256, "value": 1e5, "ms_per_step": 7.0, "steps": 20, "results_ok_steps": True,
                 "source": "value"}
    assert bench.named_length_record(2e5, 7.5, 1024, 1024, 1, 2, True, True,
                                     {"same_as_value": True, "note": ""}, 5)["source"] == "value"
    ss = {"value": 1.4e5, "ms_per_step": 5.1, "steps": 5, "content_chars": 256, "results_ok_steps": True}
    r = bench.named_length_record(8e5, 7.2, 2048, 256, 1, 8, False, True, ss, 5)
    assert r == {"chars": 256, "value": 1.4e5, "ms_per_step": 5.1, "steps": 5, "results_ok_steps": True,
                 "source": "strong_starts"}
    assert bench.named_length_record(8e5, 7.2, 2048, 256, 1, 8, False, True, None, 5) is None
    assert bench.named_length_record(8e5, 7.2, 256, 256, 8, 1, False, True, None, 5) is None  # M matches


def test_energy_meter_off_without_gpu():
    """the power record's meter: off (never an error) when amdsmi finds no matching GPU, as here;
    a region is watts = joules / seconds and mJ per bootstrap, null on a counter that went back"""
    import types

    import bench
    props = types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x72, pci_device_id=0)
    m = bench.EnergyMeter(props)
    assert m.h is None and m.read() is None
    assert m.region((100.0, 1.0), (112.5, 1.01), 2048) == pytest.approx(
        {"w": 1250.0, "seconds": 0.01, "mj_per_bootstrap": 12.5e3 / 2048})
    assert m.region((100.0, 1.0), (99.0, 1.01), 10) is None
    assert m.region(None, (1.0, 1.0), 10) is None


def test_nccl_device_guard():
    """Under nccl every local rank needs its own GPU (RCCL refuses two ranks on one
    device); gloo rehearsals may share one"""
    import bench
    assert bench.nccl_device_guard("nccl", 2, 1) and "one GPU per rank" in bench.nccl_device_guard("nccl", 2, 1)
    assert bench.nccl_device_guard("nccl", 8, 8) is None
    assert bench.nccl_device_guard("gloo", 4, 1) is None


def test_nccl_ranks_beyond_devices_exit_nonzero():
    """`--gpus 2` under nccl where fewer GPUs are visible (here: none) ends every rank
    with the guard's message and a non-zero status, before any collective"""
    res = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, timeout=240, env=_env())
    assert res.returncode != 0
    assert "one GPU per rank" in res.stderr
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]


def test_job_timeout_kills_stuck_ranks(tmp_path):
    """--job-timeout: spawned ranks that outlive it are killed as a process group and the
    launcher exits 124 (a stuck collective does not hold the node)"""
    import bench
    stub = tmp_path / "sleeper.py"
    stub.write_text("import time\ntime.sleep(600)\n")
    import time
    t = time.time()
    rc = bench.spawn_ranks(2, [], 3.0, script=str(stub))
    assert rc == 124 and time.time() - t < 120


@pytest.mark.gpu
def test_one_rank_rccl_group_pipeline():
    """The N > 1 start-shard pipeline over a one-rank RCCL group on the GPU (bench.py
    --one-rank-group): process group, stream-ordered export, device all_gather, the OR on
    rank 0 and the all-reduces run, and every step's OR decrypts to the expected bit."""
    res = subprocess.run([sys.executable, BENCH, "--one-rank-group", "--steps", "3", "--warmup", "1", "--cpu-sample", "0",
                          "--inflight", "0", "--faithful-steps", "0", "--fresh-steps", "0", "--probe=", "--saturate", "0",
                          "--weak-matches-steps", "2"], capture_output=True, text=True, timeout=300, env=_env())
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["shard"] == "starts" and "RCCL" in d["config"]["parallelism"]
    assert d["results_ok_steps"] is True and d["result_decrypted"] == d["result_expected"] == [1]
    assert len(d["per_rank"]) == 1 and d["weak_matches"]["results_ok_ranks"] == 1
    assert d["named_length"]["chars"] == 256 and d["named_length"]["value"] == d["value"]


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [0, 1])
def test_two_gloo_ranks_config4_named_length(parts):
    """BASELINE config 4 at N = 2 (two gloo ranks sharing the box's GPU): `value` is measured on
    the named 1,024 characters split by start offsets (strong scaling), one JSON line, every
    step's OR decrypting to the expected bit, both ranks reporting; with each rank's parts
    (--start-parts 0: 16 // 2 = 8, fr_has_match_parts) and with one boolean per rank (1)"""
    res = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--workload", "config4",
                          "--steps", "2", "--warmup", "1", "--weak-matches-steps", "0", "--probe=", "--saturate", "0",
                          "--start-parts", str(parts), "--job-timeout", "280"], capture_output=True, text=True,
                         timeout=300, env=_env())
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["content_chars"] == 1024 and d["scaling"] == "strong"
    assert d["config"]["shard"] == "starts" and d["results_ok_steps"] is True
    assert d["result_decrypted"] == d["result_expected"] == [1]
    assert d["config"]["start_parts"] == (parts or 8)
    assert len(d["per_rank"]) == 2 and d["strong_starts"] == {"same_as_value": True,
                                                              "note": d["strong_starts"]["note"]}
    assert d["named_length"]["source"] == "value" and d["named_length"]["chars"] == 1024
    assert d["named_length"]["value"] == d["value"] and d["named_length"]["results_ok_steps"] is True
