#!/bin/bash
# The latency shape's key prefetch re-checked under the adopted scheduler settings
# (build_variant.sh NAME -D...): ref3 = default (FR_LAT_PF=2: groups 0-1 a step ahead, group 2 at
# the top of the step); pf3 = all three groups a step ahead (222 VGPRs); pf1 = group 0 ahead.
# Three interleaved rounds of launch times (tools/lat_probe.py) and /abc/ x 256 match times.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06ab
mkdir -p $out
for r in 1 2 3; do
  for v in ref3 pf3 pf1; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
