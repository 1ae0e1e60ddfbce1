#!/bin/bash
# Interleaved A/B of environment settings on the current library: blind-rotation launch times,
# keyswitch by fan-in and the match.   bash tools/ab_env_r04.sh ROUNDS "ENV1" "ENV2" ...  ("-" = none)
set -o pipefail
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for e in "$@"; do
    [ "$e" = "-" ] && e=""
    echo "# env: ${e:-default}"
    env $e timeout -k 10 120 python3 tools/lat_probe.py 5 ${SIZES:-1 254 512 2048} || exit 1
    env $e timeout -k 10 120 python3 tools/match_ab.py 7 || exit 1
  done
done
