#!/bin/bash
# Segment timing of the blind rotation (FR_BR_TIMING builds from tools/build_variant.sh).
set -o pipefail
cd "$(dirname "$0")/.."
for v in timing timing_nobsk nobsk; do
  echo "== $v"
  FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 120 python3 tools/br_timing.py 1 256 512 || exit 1
done
