#!/bin/bash
# Interleaved A/B of library variants at the k = 2, N = 1024 point: bash tools/ab_k2.sh ROUNDS LIB...
set -o pipefail
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for lib in "$@"; do
    FR_PARAMS=k2n1024 FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 7 1 16 254 512 || exit 1
  done
done
