#!/bin/bash
# Round-4 GPU iteration: parity tests (optionally a -k filter), the default N=1 bench
# line, and the launcher-free two-rank start-shard line (gloo: both ranks share the
# box's one GPU).   bash tools/gpu_r04.sh OUTDIR [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/r04}
mkdir -p "$out"
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$out/gpu_tests.log" 2>&1 || { tail -60 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { cat "$out/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); r=d['roofline']
print('match_ms=%.3f value=%.0f frac=%.3f fresh=%s' % (d['match_ms'], d['value'], r['frac'], d['fresh_content']['fresh_content_ms']))
print('probe', {k: round(v['br_ms'],3) for k, v in d['latency_probe'].items()}, 'sat', round(d['kernel_saturated']['br_pbs_per_s']))
print('faithful', d['faithful']); print('cpu identical', d['cpu_baseline']['cpu_gpu_bit_identical'], d['cpu_baseline']['match'])
for k, v in r['per_shape'].items(): print(k, v)"
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > "$out/bench_2rank_gloo.json" 2> "$out/bench_2rank_gloo.err" || { tail -30 "$out/bench_2rank_gloo.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench_2rank_gloo.json'))
print('n_gpus', d['n_gpus'], 'shard', d['config']['shard'], 'ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'], d['result_expected'])
print('per_rank', d['per_rank']); print('weak_matches', d['weak_matches'])"
