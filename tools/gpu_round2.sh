#!/bin/bash
# Round-2 GPU check: parity tests, smoke, default bench line, a 2-rank rehearsal
# of the N>1 paths on the one GPU (gloo collectives, strong and weak), and the
# profile passes.   bash tools/gpu_round2.sh OUTDIR [no-prof]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/r2}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
step 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
step 200 python __graft_entry__.py smoke > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
step 300 python3 bench.py --steps 20 --warmup 5 --probe 1,16,254,512 > "$out/bench.json" 2> "$out/bench.err" || { cat "$out/bench.err"; exit 1; }
cat "$out/bench.json"
for mode in strong weak; do
  step 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --scaling $mode --saturate 0 > "$out/bench_2rank_gloo_$mode.json" 2> "$out/bench_2rank_gloo_$mode.err" || { tail -30 "$out/bench_2rank_gloo_$mode.err"; exit 1; }
  tail -1 "$out/bench_2rank_gloo_$mode.json"
done
[ "$2" = "no-prof" ] && exit 0
bash tools/profile.sh "$out/prof"
