#!/bin/bash
# Pair key-load placement, third round around FR_PAIR_PF=1 FR_PAIR_LOAD2=4, with matches.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04w; mkdir -p $out
E=fhe-regex_amd/build/exp
for r in 1 2 3; do
  for lib in fhe-regex_amd/libfheregex.so $E/lib_p1b4.so $E/lib_p2l4.so $E/lib_p1l1b4.so $E/lib_p1l0b4.so $E/lib_p1l4b4.so $E/lib_p2l3.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 512 2048 >> $out/lat.log 2>&1 || exit 1
  done
  for lib in fhe-regex_amd/libfheregex.so $E/lib_p1b4.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/match_ab.py 9 >> $out/lat.log 2>&1 || exit 1
  done
done
echo done
