#!/bin/bash
# Round-3 second-session GPU pass: parity tests, smoke, keyswitch A/B (workgroup order,
# k-steps in flight), the default bench line and a kernel trace.
#   bash tools/gpu_s2.sh OUTDIR [skip-tests]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/s2}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
if [ "$2" != "skip-tests" ]; then
  step 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
  tail -3 "$out/gpu_tests.log"
  step 200 python __graft_entry__.py smoke > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
  tail -1 "$out/smoke.log"
fi
for r in 1 2; do
  for v in 0 1; do
    FR_KS_XCD=$v step 120 python3 tools/ks_probe.py 9 1 17 254 512 >> "$out/ks_ab.log" 2>&1 || { cat "$out/ks_ab.log"; exit 1; }
  done
  for lib in ${KS_LIBS:-}; do
    FHEREGEX_LIB=$lib step 120 python3 tools/ks_probe.py 9 1 17 254 512 >> "$out/ks_ab.log" 2>&1 || { cat "$out/ks_ab.log"; exit 1; }
  done
done
cat "$out/ks_ab.log"
step 300 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { cat "$out/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); r=d['roofline']
print('match_ms=%.3f value=%.0f fresh=%s' % (d['match_ms'], d['value'], d['fresh_content']['fresh_content_ms']))
print('probe', {k: round(v['br_ms'],3) for k, v in d['latency_probe'].items()}, 'sat', round(d['kernel_saturated']['br_pbs_per_s']))"
step 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --saturate 0 > "$out/trace.log" 2>&1
echo done
