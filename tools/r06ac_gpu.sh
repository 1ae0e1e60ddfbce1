#!/bin/bash
# The pair shape's key-load placement re-checked under the adopted settings (build_variant.sh
# NAME -D...): ref4 = default (FR_PAIR_LOAD=2, FR_PAIR_LOAD2=4); l1 / l3 = the second group after
# forward phase 1 / 3; l2b = the third group after phase 3.
# Three interleaved rounds of launch times (tools/lat_probe.py) and /abc/ x 256 match times.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06ac
mkdir -p $out
for r in 1 2 3; do
  for v in ref4 l1 l3 l2b; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 512 2048 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
