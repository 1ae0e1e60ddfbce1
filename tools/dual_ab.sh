#!/bin/bash
# A/B of the dual-polynomial latency shape: bash tools/dual_ab.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/dual}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --probe 1,16,254,512 > "$out/$tag.json" 2> "$out/$tag.err" || { cat "$out/$tag.err"; exit 1; }; python3 -c "
import json; d=json.load(open('$out/$tag.json')); p=d.get('latency_probe') or {}
print('$tag', 'match_ms=%.3f'%d['match_ms'], 'frac=%.3f'%d['roofline']['frac'], 'sat=%.0f'%d['kernel_saturated']['br_pbs_per_s'], {k:round(v['br_ms'],3) for k,v in p.items()})"; }
run old FR_FFT_DUAL=0
run pre3 FR_X=1
run pre2 FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_pre2.so
run pre4 FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_pre4.so
