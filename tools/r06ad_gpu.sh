#!/bin/bash
# Two latency-shape knobs re-checked under the adopted scheduler settings (build_variant.sh
# NAME -D...): ref5 = default; twsgpr = wave-uniform twiddles in SGPRs (-DFR_TW_SGPR_LAT=1, 5%
# slower in round 4); prio = static priority for waves 4-7 (-DFR_PRIO_HALF_LAT=1, no change in round 6).
# Three interleaved rounds of launch times (tools/lat_probe.py) and /abc/ x 256 match times.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06ad
mkdir -p $out
for r in 1 2 3; do
  for v in ref5 twsgpr prio; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
