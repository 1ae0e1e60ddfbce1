#!/bin/bash
# The N > 1 start-shard pipeline over a ONE-rank RCCL group on the one-GPU box: process group
# init (nccl = RCCL), stream-ordered export + event, all_gather_into_tensor on device, the OR
# launch on rank 0, the max/sum all_reduces -- the collective path the driver's 8-GPU run takes.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r04i; mkdir -p $out
A="--one-rank-group --steps 10 --warmup 2 --cpu-sample 0 --inflight 0 --faithful-steps 0 --fresh-steps 0 --probe= --saturate 0"
timeout -k 10 300 python3 bench.py $A > $out/rccl1_direct.json 2> $out/rccl1_direct.log &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 $A --weak-matches-steps 5 > $out/rccl1_torchrun.json 2> $out/rccl1_torchrun.log &&
timeout -k 10 300 python3 bench.py $A --workload config4 --steps 4 > $out/rccl1_config4.json 2> $out/rccl1_config4.log &&
echo done
