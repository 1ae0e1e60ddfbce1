#!/bin/bash
# Round-3 GPU iteration: parity tests (optionally a -k filter), the default bench
# line, and the batched-throughput line.   bash tools/gpu_r03.sh OUTDIR [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/r03}
mkdir -p "$out"
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$out/gpu_tests.log" 2>&1 || { tail -60 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { cat "$out/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); r=d['roofline']
print('match_ms=%.3f value=%.0f frac=%.3f fresh=%s' % (d['match_ms'], d['value'], r['frac'], d['fresh_content']['fresh_content_ms']))
print('probe', {k: round(v['br_ms'],3) for k, v in d['latency_probe'].items()}, 'sat', round(d['kernel_saturated']['br_pbs_per_s']))
print('shapes', r['per_shape'])"
for M in 8 16; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --matches $M --cpu-sample 0 --probe '' --fresh-steps 0 --saturate 0 > "$out/bench_m$M.json" 2> "$out/bench_m$M.err" || { cat "$out/bench_m$M.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/bench_m$M.json')); print('M=$M', 'step_ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'])"
done
