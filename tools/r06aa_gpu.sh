#!/bin/bash
# A/B of generic machine-scheduler knobs on top of the adopted settings (trackers everywhere,
# max-ILP for the pair TU), applied to every TU by build_variant.sh NAME FLAGS:
#   ref2       the default build
#   nocluster  -mllvm --misched-cluster=false
#   postra     -mllvm --misched-postra
#   topdown    -mllvm --misched-prera-direction=topdown
#   bottomup   -mllvm --misched-prera-direction=bottomup
# Three interleaved rounds of launch times (tools/lat_probe.py) and /abc/ x 256 match times.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06aa
mkdir -p $out
for r in 1 2 3; do
  for v in ref2 nocluster postra topdown bottomup; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 512 2048 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
