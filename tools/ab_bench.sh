#!/bin/bash
# A/B of kernel variants on one box: saturated PBS throughput + /abc/ x256 e2e.
set -o pipefail
cd "$(dirname "$0")/.."
run() { echo "== $1"; shift; timeout -k 10 300 env "$@" python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --probe 1,64,256,512,1024 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_saturated']
print(' '.join('%d:%.2fms' % (int(c), v['br_ms']) for c, v in (d['latency_probe'] or {}).items()))
print('e2e %.0f rot/s  match %.1f ms  rot %d  luts %d  levels %d  br_avg %.2f ms/launch  saturated %.0f PBS/s (br %.1f ms / %d)' % (d['value'], d['ms_per_step'], d['blind_rotations_per_match'], d['lut_outputs_per_match'], d['levels'], d['roofline']['br_avg_ms'], k['pbs_per_s'], k['br_ms_per_launch'], k['gates_per_launch']))"; }
for v in "$@"; do run "$v" $v || exit 1; done
