#!/bin/bash
# A/B of the AMDGPU machine scheduler on the blind-rotation kernels (same source, same
# arithmetic: scheduling does not change a rounding, so every variant is bit-exact):
#   base     the default (GCN max-occupancy scheduler)
#   maxilp   -mllvm --amdgpu-sched-strategy=max-ilp            (latency 255 / pair 255 VGPRs)
#   maxmem   -mllvm --amdgpu-sched-strategy=max-memory-clause  (217 / 252)
#   iterilp  -mllvm --amdgpu-sched-strategy=iterative-ilp      (235 / 254)
# built by tools/build_variant.sh NAME FLAGS.  Three interleaved rounds of launch times
# (tools/lat_probe.py) and of /abc/ x 256 match times (tools/match_ab.py).
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06v
mkdir -p $out
for r in 1 2 3; do
  for v in base maxilp maxmem iterilp; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 512 2048 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
