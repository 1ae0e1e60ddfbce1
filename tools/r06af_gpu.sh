#!/bin/bash
# The k = 2, N = 1024 point (BASELINE config 2's "N=1024" parameters) under the scheduler
# strategies (build_variant.sh NAME -mllvm --amdgpu-sched-strategy=..., every TU; the k = 2
# kernels are the latency shape E = 4 and the throughput shape E = 8, both in fft_br.hip):
# ref6 = the adopted settings.  Three interleaved rounds at k = 2 of launch times and of
# /abc/ x 256 match times (FR_PARAMS=k2n1024).
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06af
mkdir -p $out
export FR_PARAMS=k2n1024
for r in 1 2 3; do
  for v in ref6 k2maxilp k2iter k2maxmem; do
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/lat_probe.py 7 1 16 254 1024 \
      >> $out/lat.log 2>&1 || { echo "FAILED lat $v"; tail -5 $out/lat.log; exit 1; }
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 150 python3 tools/match_ab.py 5 \
      >> $out/match.log 2>&1 || { echo "FAILED match $v"; tail -5 $out/match.log; exit 1; }
  done
done
cat $out/lat.log $out/match.log
