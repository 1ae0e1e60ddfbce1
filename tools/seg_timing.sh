#!/bin/bash
# Segment timing of the blind rotation (FR_BR_TIMING build from tools/build_variant.sh timing):
# s_memtime deltas of wave 0 of workgroup 0 per step segment, at 1, 256 and 512 bootstraps.
set -o pipefail
cd "$(dirname "$0")/.."
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_timing.so timeout -k 10 120 python3 tools/br_timing.py 1 256 512
