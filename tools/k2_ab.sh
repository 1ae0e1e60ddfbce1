#!/bin/bash
# k = 2, N = 1024 FFT-ring shape A/B on the GPU box: bash tools/k2_ab.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/k2ab}
mkdir -p "$out"
run() { local tag=$1; shift; echo "== $tag: $*"; env "$@" timeout -k 10 200 python3 bench.py --params k2n1024 --steps 10 --warmup 3 --cpu-sample 0 --probe 1,16,128,254,512 > "$out/$tag.json" 2> "$out/$tag.err" || { cat "$out/$tag.err"; exit 1; }; python3 -c "
import json,sys; d=json.load(open('$out/$tag.json'))
print('$tag', 'match_ms=%.3f'%d['match_ms'], 'frac=%.3f'%d['roofline']['frac'], 'sat=%.0f'%d['kernel_saturated']['br_pbs_per_s'], {k:round(v['br_ms'],3) for k,v in d['latency_probe'].items()})"; }
run default FR_X=0
run tpE4 FR_FFT_LANE_ELEMS=4
run allTP FR_FFT_SMALL_BATCH=0
run allLAT FR_FFT_SMALL_BATCH=100000
