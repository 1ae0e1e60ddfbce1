#!/bin/bash
# A/B of kernel variants on one box: saturated PBS throughput + /abc/ x256 e2e.
set -o pipefail
cd "$(dirname "$0")/.."
run() { echo "== $1"; shift; timeout -k 10 300 env "$@" python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_saturated']
print('e2e %.0f PBS/s  match %.1f ms  br_avg %.2f ms/launch  saturated %.0f PBS/s (br %.1f ms / %d)' % (d['value'], d['ms_per_step'], d['roofline']['br_avg_ms'], k['pbs_per_s'], k['br_ms_per_launch'], k['gates_per_launch']))"; }
run "E=8 default (146 VGPR)" FR_LANE_ELEMS=8 || exit 1
run "E=8 W=4 (128 VGPR)" FR_LANE_ELEMS=8 FHEREGEX_LIB=fhe-regex_amd/build/exp/libfheregex_w4.so || exit 1
run "E=16" FR_LANE_ELEMS=16 || exit 1
