#!/bin/bash
# GPU A/B pass: a parity subset at HEAD (-k expression), the interleaved A/B of library
# variants (tools/ab_r04.sh) and the default bench line.   bash tools/gpu_ab.sh OUT "K-EXPR" LIB...
set -o pipefail
cd "$(dirname "$0")/.."
out=$1; kexpr=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
step 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$kexpr" > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
step 900 bash tools/ab_r04.sh ${ROUNDS:-3} "$@" > "$out/ab.log" 2>&1 || { cat "$out/ab.log"; exit 1; }
cat "$out/ab.log"
step 400 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --faithful-steps 0 > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); r=d['roofline']
print('match_ms=%.3f value=%.0f frac=%.3f fresh=%s' % (d['match_ms'], d['value'], r['frac'], d['fresh_content']['fresh_content_ms']))
print('probe', {k: round(v['br_ms'],3) for k, v in d['latency_probe'].items()}, 'sat', round(d['kernel_saturated']['br_pbs_per_s']))"
