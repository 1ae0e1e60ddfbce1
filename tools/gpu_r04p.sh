#!/bin/bash
# Small-level digit pass (k_ks_digits16q): keyswitch + whole-match parity, then keyswitch by
# fan-in and the match with FR_KS_DIG16Q=0 / 1 interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04p; mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "keyswitch or match_words or or_each or run_gates or gates" > $out/tests.log 2>&1 &&
for r in 1 2 3; do
  for q in 0 1; do
    echo "# FR_KS_DIG16Q=$q" >> $out/ab.log
    FR_KS_DIG16Q=$q timeout -k 10 120 python3 tools/ks_fanin_probe.py 9 >> $out/ab.log 2>&1 || exit 1
    FR_KS_DIG16Q=$q timeout -k 10 120 python3 tools/match_ab.py 7 >> $out/ab.log 2>&1 || exit 1
  done
done
echo done
