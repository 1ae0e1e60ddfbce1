#!/bin/bash
# Per-workgroup start/end stamps of the blind-rotation launches (FR_WG_STAMPS variant): the
# spread of workgroup durations within a launch, by XCC.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04l; mkdir -p $out
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_stamps.so timeout -k 10 200 python3 tools/gap_probe.py off 6 > $out/match.log 2> $out/match_stamps.log &&
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_stamps.so timeout -k 10 200 python3 tools/lat_probe.py 3 1 254 512 2048 > $out/lat.log 2> $out/lat_stamps.log &&
echo done
