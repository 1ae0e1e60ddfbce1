#!/bin/bash
# Pair shape (two bootstraps per workgroup): parity, then an interleaved A/B of the
# launch times and of the /abc/ x 256 match with the shape off / on.
#   bash tools/gpu_pair.sh OUTDIR [LIMITS...]   (FR_FFT_PAIR_BATCH values; default 0 4096)
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/pair}; shift
lims=${*:-0 4096}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_fft.py -m gpu \
  -k "pair or throughput" > "$out/tests_fft.log" 2>&1 || { tail -30 "$out/tests_fft.log"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "pair_shape and fft and not k2" > "$out/tests_gpu.log" 2>&1 || { tail -30 "$out/tests_gpu.log"; exit 1; }
envs=()
for l in $lims; do envs+=("FR_FFT_PAIR_BATCH=$l"); done
SIZES="${SIZES:-257 512 1024 2048}" bash tools/ab_env.sh 2 "${envs[@]}" > "$out/ab.log" 2>&1 || { cat "$out/ab.log"; exit 1; }
cat "$out/ab.log"
for r in 1 2; do
  for l in $lims; do
    FR_FFT_PAIR_BATCH=$l timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --probe= --fresh-steps 0 \
      > "$out/bench_${l}_$r.json" 2> "$out/bench_${l}_$r.err" || { tail -20 "$out/bench_${l}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('pair<=$l', 'match_ms', round(d['match_ms'],3), 'sat', round(d['kernel_saturated']['br_pbs_per_s']))" "$out/bench_${l}_$r.json"
  done
done
