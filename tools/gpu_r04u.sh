#!/bin/bash
# Key-load placement re-check at HEAD: pair (FR_PAIR_LOAD, FR_PAIR_PF) and latency (FR_LAT_LOAD1, FR_LAT_PF) variants.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04u; mkdir -p $out
E=fhe-regex_amd/build/exp
for r in 1 2 3; do
  for lib in fhe-regex_amd/libfheregex.so $E/lib_pl1.so $E/lib_pl3.so $E/lib_ppf1.so $E/lib_ll1.so $E/lib_ll3.so $E/lib_lpf1.so $E/lib_lpf3.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 1 254 512 2048 >> $out/lat.log 2>&1 || exit 1
  done
done
echo done
