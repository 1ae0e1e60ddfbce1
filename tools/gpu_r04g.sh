#!/bin/bash
# Two-rank gloo rehearsal of --scaling strong --shard starts (fixed content, start offsets split).
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04g; mkdir -p $out
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --scaling strong --shard starts --steps 6 --warmup 1 --cpu-sample 0 --faithful-steps 0 --fresh-steps 0 --weak-matches-steps 0 --inflight 0 --probe= > $out/strong_starts_2.json 2> $out/strong_starts_2.log &&
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --workload config4 --scaling strong --shard starts --steps 4 --warmup 1 --cpu-sample 0 --faithful-steps 0 --fresh-steps 0 --weak-matches-steps 0 --inflight 0 --probe= > $out/strong_starts_2_config4.json 2> $out/strong_starts_2_config4.log &&
echo done
