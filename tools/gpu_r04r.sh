#!/bin/bash
# Timing-only builds (wrong results): what the LDS exchanges cost in the pair and latency shapes.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04r; mkdir -p $out
for r in 1 2; do
  for lib in fhe-regex_amd/libfheregex.so fhe-regex_amd/build/exp/lib_noxchg.so fhe-regex_amd/build/exp/lib_nocross.so fhe-regex_amd/build/exp/lib_nolocal.so fhe-regex_amd/build/exp/lib_nomacx.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 1 254 512 2048 >> $out/lat.log 2>&1 || exit 1
  done
done
echo done
