#!/bin/bash
# The pair shape under the max-ILP scheduler (fft_br_pair.hip, Makefile PAIR_SCHED) as the
# default: the full GPU suite through it, then three interleaved A/B rounds against the same
# source with the default scheduler for the pair TU (build_variant.sh pairdef, PAIR_SCHED="").
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06w
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 \
  || { echo "FAILED tests"; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for r in 1 2 3; do
  for v in pairdef new; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 512 2048 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
