#!/bin/bash
# One GPU-box recipe for every measurement of this repository (replaces the per-iteration
# gpu_r0N*.sh scripts).  Every GPU step runs under its own time limit; the script stops at
# the first failure and prints the tail of that step's log.
#   bash tools/gpu_run.sh OUTDIR PARTS [pytest -k expr]
# PARTS: comma-separated, run in the order given:
#   tests      pytest -m gpu (the -k expr, if given, selects)
#   smoke      __graft_entry__ smoke
#   ubench     tools/ubench_keystream (key-stream rate per CU; built here on the CPU)
#   profile    tools/profile.sh: rocprofv3 kernel trace + PMC passes -> OUTDIR/prof/pmc_summary.json
#   bench      the default N = 1 bench line (20 steps; with OUTDIR/prof/pmc_summary.json if profiled)
#   batch      M = 8 / 16 matches per step
#   workloads  one N = 1 line per BASELINE workload (and the k = 2, N = 1024 point)
#   rehearsal  launcher-free two-rank lines (gloo, both ranks on the box's one GPU): the metric
#              default (weak start shards + strong_starts), config 4's default (1,024 chars split
#              by start offsets), config 5's default (closure shards), weak by matches
#   rehearsal4 the same with four gloo ranks (the metric and config 4; 16 // 4 = 4 parts per rank)
#   rccl1      the N > 1 start-shard pipeline over a one-rank RCCL group
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:?OUTDIR}
parts=${2:?PARTS}
kexpr=${3:-}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1 log=$2; shift 2; echo "== $*" >&2; timeout -k 10 "$t" "$@" > "$log" 2>&1 || { rc=$?; echo "step failed rc=$rc: $*"; tail -40 "$log"; exit 1; }; }
summ() { python3 tools/bench_summary.py "$@"; }
IFS=',' read -ra P <<< "$parts"
for part in "${P[@]}"; do
  case $part in
  tests)
    K=(); [ -n "$kexpr" ] && K=(-k "$kexpr")
    step 1100 "$out/gpu_tests.log" python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${K[@]}"
    tail -1 "$out/gpu_tests.log" ;;
  smoke)
    step 200 "$out/smoke.log" python __graft_entry__.py smoke
    tail -1 "$out/smoke.log" ;;
  ubench)
    step 300 "$out/ubench_keystream.log" ./tools/ubench_keystream
    cat "$out/ubench_keystream.log" ;;
  profile)
    step 1000 "$out/profile.log" bash tools/profile.sh "$out/prof"
    tail -2 "$out/profile.log" ;;
  bench)
    pmc=(); [ -f "$out/prof/pmc_summary.json" ] && pmc=(--pmc "$out/prof/pmc_summary.json")
    step 500 "$out/bench.err" python3 bench.py --steps 20 --warmup 5 "${pmc[@]}" --out "$out/bench.json"
    summ "$out/bench.json" ;;
  batch)
    for M in 8 16; do
      step 300 "$out/bench_m$M.err" python3 bench.py --steps 5 --warmup 2 --matches $M --cpu-sample 0 --probe= \
        --fresh-steps 0 --saturate 0 --faithful-steps 0 --faithful-tree-steps 0 --out "$out/bench_m$M.json"
      summ "$out/bench_m$M.json"
    done ;;
  workloads)
    for w in "config2 --params k2n1024" "config2" "metric --params k2n1024" "config3" "config4" "config5"; do
      tag=$(echo $w | tr -d ' -')
      step 400 "$out/bench_$tag.err" python3 bench.py --workload $w --steps 5 --warmup 2 --cpu-sample 0 --saturate 0 \
        --faithful-steps 0 --faithful-tree-steps 0 --out "$out/bench_$tag.json"
      summ "$out/bench_$tag.json"
    done ;;
  rehearsal)
    for mode in "metric" "config4" "config5" "metric --shard matches"; do
      tag=$(echo $mode | sed 's/ --shard /_/')
      step 500 "$out/rehearsal_2rank_$tag.err" python3 bench.py --gpus 2 --dist-backend gloo --workload $mode \
        --steps 5 --warmup 1 --out "$out/rehearsal_2rank_$tag.json"
      summ "$out/rehearsal_2rank_$tag.json"
    done ;;
  rehearsal4)
    for mode in metric config4; do
      step 600 "$out/rehearsal_4rank_$mode.err" python3 bench.py --gpus 4 --dist-backend gloo --workload $mode \
        --steps 3 --warmup 1 --saturate 0 --probe= --out "$out/rehearsal_4rank_$mode.json"
      summ "$out/rehearsal_4rank_$mode.json"
    done ;;
  rccl1)
    step 300 "$out/rccl1.err" python3 bench.py --one-rank-group --steps 10 --warmup 2 --cpu-sample 0 --inflight 0 \
      --faithful-steps 0 --faithful-tree-steps 0 --out "$out/rccl1.json"
    summ "$out/rccl1.json" ;;
  *) echo "unknown part $part"; exit 2 ;;
  esac
done
echo done
