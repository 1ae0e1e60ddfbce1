#!/bin/bash
# Noise at both FFT points and one bench line per BASELINE workload (N = 1):
#   bash tools/workloads.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/wl}
mkdir -p "$out"
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
step 300 python3 tools/noise.py 1024 "$out/noise_k1n2048.json" > /dev/null
FR_PARAMS=k2n1024 step 300 python3 tools/noise.py 1024 "$out/noise_k2n1024.json" > /dev/null
for w in "config2 --params k2n1024" "config2" "metric --params k2n1024" "config3" "config4" "config5"; do
  tag=$(echo $w | tr -d ' -')
  step 400 python3 bench.py --workload $w --steps 5 --warmup 2 --cpu-sample 0 --saturate 0 > "$out/bench_$tag.json" 2> "$out/bench_$tag.err" || { tail -20 "$out/bench_$tag.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/bench_$tag.json'))
print('$tag', d['config']['workload'], d['config']['params'], 'match_ms=%.2f'%d['match_ms'], 'rot=%d'%d['blind_rotations_per_step'], 'levels=%d'%d['levels'], 'value=%.0f'%d['value'], 'frac=%.3f'%d['roofline']['frac'], 'ok=%s'%(d['result_decrypted']==d['result_expected']))"
done
