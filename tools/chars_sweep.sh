#!/bin/bash
# /abc/ match time against content length on one GPU:  bash tools/chars_sweep.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/chars}
mkdir -p "$out"
export TMPDIR=/tmp
for c in 64 256 1024 2048 4096; do
  timeout -k 10 300 python3 bench.py --chars $c --steps 3 --warmup 1 --cpu-sample 0 --saturate 0 --probe '' --fresh-steps 0 --faithful-steps 0 --inflight 0 > "$out/abc_$c.json" 2> "$out/abc_$c.err" || { tail -20 "$out/abc_$c.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/abc_$c.json'))
print('chars=$c', 'match_ms=%.2f' % d['match_ms'], 'rot=%d' % d['blind_rotations_per_step'], 'levels=%d' % d['levels'], 'value=%.0f' % d['value'], d['result_decrypted'], d['result_expected'])"
done
