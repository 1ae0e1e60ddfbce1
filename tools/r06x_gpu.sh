#!/bin/bash
# A/B of further AMDGPU scheduling knobs on every kernel (after the pair TU's max-ILP split;
# build_variant.sh NAME FLAGS applies FLAGS to device.hip, fft_br.hip and fft_br_pair.hip):
#   ref        the default build
#   bias0      -mllvm --amdgpu-schedule-metric-bias=0
#   bias100    -mllvm --amdgpu-schedule-metric-bias=100
#   nounclust  -mllvm --amdgpu-disable-unclustered-high-rp-reschedule
#   trackers   -mllvm --amdgpu-use-amdgpu-trackers
# Three interleaved rounds of launch times (tools/lat_probe.py) and /abc/ x 256 match times.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06x
mkdir -p $out
for r in 1 2 3; do
  for v in ref bias0 bias100 nounclust trackers; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 512 2048 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
