#!/bin/bash
# Round-4 closing GPU pass at HEAD: parity tests, smoke, rocprofv3 trace + PMC passes
# (tools/profile.sh), the default bench line, batched lines, one line per BASELINE
# workload, and the launcher-free two-rank rehearsals (gloo, ranks sharing the GPU).
#   bash tools/final_r04.sh OUTDIR [all|a|b|p]   (a: tests, smoke, profile, bench line; b: the rest;
#   p: profile and bench line only)
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/final_r04}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
part=${2:-all}
if [ "$part" != "b" ] && [ "$part" != "p" ]; then
  step 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
  tail -1 "$out/gpu_tests.log"
  step 200 python __graft_entry__.py smoke > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
  tail -1 "$out/smoke.log"
fi
if [ "$part" != "b" ]; then
step 900 bash tools/profile.sh "$out/prof" > "$out/profile.log" 2>&1 || { tail -20 "$out/profile.log"; exit 1; }
step 400 python3 bench.py --steps 20 --warmup 5 --pmc "$out/prof/pmc_summary.json" > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print('match_ms=%.3f value=%.0f fresh=%.3f frac=%.3f' % (d['match_ms'], d['value'], d['fresh_content']['fresh_content_ms'], d['roofline']['frac']))
print('probe', {k: round(v['br_ms'],3) for k, v in d['latency_probe'].items()}, 'sat', round(d['kernel_saturated']['br_pbs_per_s']))"
fi
[ "$part" = "a" ] || [ "$part" = "p" ] && { echo done; exit 0; }
for M in 8 16; do
  step 300 python3 bench.py --steps 5 --warmup 2 --matches $M --cpu-sample 0 --probe '' --fresh-steps 0 --saturate 0 --faithful-steps 0 > "$out/bench_m$M.json" 2> "$out/bench_m$M.err" || { tail -20 "$out/bench_m$M.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/bench_m$M.json')); print('M=$M', 'step_ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'])"
done
for w in "config2 --params k2n1024" "config2" "metric --params k2n1024" "config3" "config4" "config5"; do
  tag=$(echo $w | tr -d ' -')
  step 400 python3 bench.py --workload $w --steps 5 --warmup 2 --cpu-sample 0 --saturate 0 --faithful-steps 0 > "$out/bench_$tag.json" 2> "$out/bench_$tag.err" || { tail -20 "$out/bench_$tag.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/bench_$tag.json'))
print('$tag', d['config']['workload'], d['config']['params'], 'match_ms=%.2f'%d['match_ms'], 'rot=%d'%d['blind_rotations_per_step'], 'levels=%d'%d['levels'], 'value=%.0f'%d['value'], 'ok=%s'%(d['result_decrypted']==d['result_expected']))"
done
for mode in "--scaling weak --shard starts" "--scaling weak --shard matches" "--scaling strong --shard closure"; do
  tag=$(echo $mode | sed 's/--scaling //; s/ --shard /_/')
  step 400 python3 bench.py --gpus 2 --dist-backend gloo $mode --steps 10 --warmup 2 > "$out/rehearsal_2rank_$tag.json" 2> "$out/rehearsal_2rank_$tag.err" || { tail -30 "$out/rehearsal_2rank_$tag.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/rehearsal_2rank_$tag.json'))
print('2 ranks $tag', 'ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'], d['result_expected'], d.get('results_ok_steps'))"
done
echo done
