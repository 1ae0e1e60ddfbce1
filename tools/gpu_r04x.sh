#!/bin/bash
# Fourth placement round: pair cc / twiddle registers, latency third group before the MAC.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04x; mkdir -p $out
E=fhe-regex_amd/build/exp
for r in 1 2 3; do
  for lib in fhe-regex_amd/libfheregex.so $E/lib_cc0.so $E/lib_twv.so $E/lib_lt4.so $E/lib_lt3.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 1 16 254 512 2048 >> $out/lat.log 2>&1 || exit 1
  done
done
echo done
