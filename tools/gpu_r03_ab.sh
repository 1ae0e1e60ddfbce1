#!/bin/bash
# A/B of library variants (single-bootstrap and batch latency), then the round-3 iteration.
#   bash tools/gpu_r03_ab.sh OUTDIR LIB...
set -o pipefail
cd "$(dirname "$0")/.."
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/ab_libs.sh 2 "$@" > "$out/ab.log" 2>&1 || { cat "$out/ab.log"; exit 1; }
cat "$out/ab.log"
bash tools/gpu_r03.sh "$out"
