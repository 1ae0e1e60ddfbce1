#!/bin/bash
# Round-end measurement on one GPU box: profile passes, PMC summary, noise,
# and the default bench line (reads profiles/$R/pmc_summary.json for traffic).
#   bash tools/round_measure.sh r01
set -o pipefail
cd "$(dirname "$0")/.."
R=${1:-r01}
out=gpurun_out/prof_$R
bash tools/profile.sh "$out" || exit 1
python3 tools/pmc_summary.py "$out" "$out/pmc_summary.json" || exit 1
mkdir -p profiles/$R && cp "$out/pmc_summary.json" profiles/$R/pmc_summary.json
timeout -k 10 300 python3 tools/noise.py 256 "$out/noise.json" > "$out/noise.log" 2>&1 || { echo "noise failed"; exit 1; }
timeout -k 10 600 python3 bench.py > "$out/bench_default.jsonl" 2> "$out/bench_default.err" || { echo "bench failed"; exit 1; }
tail -1 "$out/bench_default.jsonl"
