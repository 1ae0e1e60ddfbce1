#!/bin/bash
# Launch gaps with the event timers on / off (kernel traces) and the match's wall time both ways.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r04j; mkdir -p $out
timeout -k 10 200 python3 tools/match_probe.py 15 > $out/match_probe.log 2>&1 &&
timeout -k 10 120 tools/ubench_gap > $out/ubench_gap.log 2>&1 &&
for m in off on all; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $out/gap_$m -o run --output-format csv -- python3 tools/gap_probe.py $m 10 > $out/gap_$m.log 2>&1 || exit 1
done
echo done
