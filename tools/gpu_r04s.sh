#!/bin/bash
# Pair-shape offset schedule (FR_PAIR_OFS variant): pair parity, then launch times and the match vs HEAD.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04s; mkdir -p $out
V=fhe-regex_amd/build/exp/lib_${1:-ofs}.so
FHEREGEX_LIB=$V timeout -k 10 400 python3 -u -m pytest tests/test_fft.py tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "pair_shape or (full_size_configs and metric)" > $out/tests.log 2>&1 &&
for r in 1 2 3; do
  for lib in fhe-regex_amd/libfheregex.so $V; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 512 2048 >> $out/ab.log 2>&1 || exit 1
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/match_ab.py 7 >> $out/ab.log 2>&1 || exit 1
  done
done
echo done
