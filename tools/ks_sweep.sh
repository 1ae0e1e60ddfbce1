#!/bin/bash
# keyswitch settings sweep on one box (tools/ks_probe.py per setting)
set -o pipefail
cd "$(dirname "$0")/.."
for v in "FR_KS_SPLIT=0" "FR_KS_SPLIT=4" "FR_KS_SPLIT=8" "FR_KS_MC=2"; do
  env $v timeout -k 10 120 python3 tools/ks_probe.py 9 1 17 254 512 || exit 1
done
