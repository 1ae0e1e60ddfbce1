#!/bin/bash
# Interleaved A/B of library variants on one box: bash tools/ab_libs.sh ROUNDS LIB...
# (each LIB a path to a libfheregex.so variant, tools/build_variant.sh)
set -o pipefail
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for lib in "$@"; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 7 ${SIZES:-} || exit 1
  done
done
