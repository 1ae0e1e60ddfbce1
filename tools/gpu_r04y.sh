#!/bin/bash
# Pair psi lookups ahead of the MAC barrier on the new key placement.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04y; mkdir -p $out
E=fhe-regex_amd/build/exp
for r in 1 2 3; do
  for lib in fhe-regex_amd/libfheregex.so $E/lib_psie.so $E/lib_psie2.so; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 512 2048 >> $out/lat.log 2>&1 || exit 1
  done
done
echo done
