#!/bin/bash
# The two remaining scheduler strategies on every TU (build_variant.sh NAME -mllvm
# --amdgpu-sched-strategy=...; the variant's strategy also replaces the pair TU's max-ILP):
# ref7 = the adopted settings; minreg = iterative-minreg; maxocc = iterative-maxocc.
# Three interleaved rounds of launch times (tools/lat_probe.py) and /abc/ x 256 match times.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06ag
mkdir -p $out
for r in 1 2 3; do
  for v in ref7 minreg maxocc; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
