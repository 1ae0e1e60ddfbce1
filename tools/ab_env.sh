#!/bin/bash
# Interleaved A/B of one library under environment settings on one box:
#   bash tools/ab_env.sh ROUNDS "VAR=a" "VAR=b" ...   (each argument: space-separated assignments, or "-")
set -o pipefail
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then e=""; fi
    echo -n "[$e] "
    env $e timeout -k 10 120 python3 tools/lat_probe.py 7 ${SIZES:-} || exit 1
  done
done
