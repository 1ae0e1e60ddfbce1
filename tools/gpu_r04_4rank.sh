#!/bin/bash
# Four launcher-free gloo ranks sharing the box's one GPU: the start-shard default and the
# strong closure mode at N = 4 (a correctness rehearsal of the N > 1 logic, not a speed figure).
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/r04_4rank}; mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
for mode in "--scaling weak --shard starts" "--scaling strong --shard closure"; do
  tag=$(echo $mode | sed 's/--scaling //; s/ --shard /_/')
  step 500 python3 bench.py --gpus 4 --dist-backend gloo $mode --steps 6 --warmup 1 > "$out/rehearsal_4rank_$tag.json" 2> "$out/rehearsal_4rank_$tag.err" || { tail -30 "$out/rehearsal_4rank_$tag.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/rehearsal_4rank_$tag.json'))
print('4 ranks $tag', 'n_gpus', d['n_gpus'], 'ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'], d['result_expected'], d.get('results_ok_steps'), len(d['per_rank']))"
done
