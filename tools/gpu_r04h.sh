#!/bin/bash
# Digit-pass rework: keyswitch + whole-match parity, then an interleaved A/B against HEAD's library.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04h; mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "keyswitch or match_words or start_shards or export_async" > $out/tests.log 2>&1 &&
SIZES="1 16" bash tools/ab_r04.sh 3 fhe-regex_amd/build/exp/lib_head.so fhe-regex_amd/build/exp/lib_dig.so > $out/ab.log 2>&1 &&

for s in 4 8 10 20 40; do
  echo "# FR_KS_SPLIT=$s" >> $out/split.log
  FR_KS_SPLIT=$s FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_dig.so timeout -k 10 120 python3 tools/ks_fanin_probe.py 9 >> $out/split.log 2>&1 || exit 1
done
echo done
