#!/bin/bash
# On the GPU box: GPU parity tests, smoke, one default bench line and a rocprofv3
# kernel trace of a short bench.   bash tools/gpu_check.sh OUTDIR [skip-tests]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/check}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
if [ "$2" != "skip-tests" ]; then
  step 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
  tail -3 "$out/gpu_tests.log"
  step 200 python __graft_entry__.py smoke > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
  tail -1 "$out/smoke.log"
fi
step 300 python3 bench.py --steps 20 --warmup 5 > "$out/bench.jsonl" 2> "$out/bench.err" || { cat "$out/bench.err"; exit 1; }
cat "$out/bench.jsonl"
step 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --saturate 0 > "$out/trace.log" 2>&1
echo done
