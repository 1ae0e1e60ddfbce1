#!/bin/bash
# Pair key-load placement, second round (FR_PAIR_PF=1 variants) and the match with FR_PAIR_PF=1.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04v; mkdir -p $out
E=fhe-regex_amd/build/exp
for r in 1 2 3; do
  for lib in fhe-regex_amd/libfheregex.so $E/lib_ppf1.so $E/lib_p1l1.so $E/lib_p1b4.so $E/lib_p1l1b2.so $E/lib_p1l3b4.so $E/lib_p1l0b2.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 512 2048 >> $out/lat.log 2>&1 || exit 1
  done
  for lib in fhe-regex_amd/libfheregex.so $E/lib_ppf1.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/match_ab.py 9 >> $out/lat.log 2>&1 || exit 1
  done
done
echo done
