#!/bin/bash
# Keyswitch A/B on one box: the keyswitch parity tests, then tools/ks_probe.py under each
# environment setting (interleaved rounds).   bash tools/ks_ab.sh OUTDIR ROUNDS "ENV1" "ENV2" ...
# (an ENV is a space-separated list of VAR=value, or "default")
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/ks_ab}; shift
rounds=${1:-2}; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k keyswitch > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for r in $(seq "$rounds"); do
  for e in "$@"; do
    [ "$e" = default ] && e=""
    env $e timeout -k 10 120 python3 tools/ks_probe.py 9 ${KS_SIZES:-1 17 254 512} >> "$out/ks_ab.log" 2>&1 || { cat "$out/ks_ab.log"; exit 1; }
  done
done
cat "$out/ks_ab.log"
