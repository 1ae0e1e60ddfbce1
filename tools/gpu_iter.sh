#!/bin/bash
# One GPU iteration: parity tests, then the default bench line with a latency probe
# and the k = 2, N = 1024 line.   bash tools/gpu_iter.sh OUTDIR [tests-only|bench-only]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/iter}
mkdir -p "$out"
export TMPDIR=/tmp
if [ "$2" != "bench-only" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
  tail -2 "$out/gpu_tests.log"
fi
[ "$2" = "tests-only" ] && exit 0
summ() { python3 -c "
import json; d=json.load(open('$1'))
p=d.get('latency_probe') or {}
print('$1', 'match_ms=%.3f'%d['match_ms'], 'frac=%.3f'%d['roofline']['frac'], 'sat=%.0f'%d['kernel_saturated']['br_pbs_per_s'], {k:round(v['br_ms'],3) for k,v in p.items()})"; }
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --probe 1,16,254,512 > "$out/bench_k1.json" 2> "$out/bench_k1.err" || { cat "$out/bench_k1.err"; exit 1; }
summ "$out/bench_k1.json"
timeout -k 10 200 python3 bench.py --params k2n1024 --steps 20 --warmup 5 --cpu-sample 0 --probe 1,16,254,512 > "$out/bench_k2.json" 2> "$out/bench_k2.err" || { cat "$out/bench_k2.err"; exit 1; }
summ "$out/bench_k2.json"
