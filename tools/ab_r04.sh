#!/bin/bash
# Interleaved A/B of library variants: blind-rotation launch times (lat_probe), keyswitch
# by fan-in (ks_fanin_probe) and the /abc/ x 256 match (match_ab).
#   bash tools/ab_r04.sh ROUNDS LIB...
set -o pipefail
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for lib in "$@"; do
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/lat_probe.py 5 ${SIZES:-1 16 254 512 2048} || exit 1
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/ks_fanin_probe.py 7 || exit 1
    FHEREGEX_LIB=$lib timeout -k 10 120 python3 tools/match_ab.py 7 || exit 1
  done
done
