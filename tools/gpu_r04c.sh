#!/bin/bash
# Round-4 GPU pass: full parity suite, smoke, an A/B of two library builds, the N=1
# bench line and the launcher-free two-rank start-shard line.   bash tools/gpu_r04c.sh OUT LIB_A LIB_B
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/r04c}; A=$2; B=$3
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
step 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
step 200 python __graft_entry__.py smoke > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
if [ -n "$A" ]; then
  shift 1
  step 900 bash tools/ab_r04.sh 3 "$@" > "$out/ab.log" 2>&1 || { cat "$out/ab.log"; exit 1; }
  cat "$out/ab.log"
fi
step 400 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); r=d['roofline']
print('match_ms=%.3f value=%.0f frac=%.3f fresh=%s' % (d['match_ms'], d['value'], r['frac'], d['fresh_content']['fresh_content_ms']))
print('probe', {k: round(v['br_ms'],3) for k, v in d['latency_probe'].items()}, 'sat', round(d['kernel_saturated']['br_pbs_per_s']))
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['value_1t'], d['cpu_baseline']['cpu_gpu_bit_identical'], d['cpu_baseline']['match']['ms'])"
step 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > "$out/bench_2rank_gloo.json" 2> "$out/bench_2rank_gloo.err" || { tail -30 "$out/bench_2rank_gloo.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench_2rank_gloo.json'))
print('n_gpus', d['n_gpus'], 'shard', d['config']['shard'], 'ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'], d['result_expected'], d['results_ok_steps'])
print('per_rank', d['per_rank']); print('lat', d['step_latency']); print('weak_matches', d['weak_matches'])"
