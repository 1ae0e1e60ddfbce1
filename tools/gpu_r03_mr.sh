#!/bin/bash
# Two ranks sharing the one GPU of the box over gloo (a rehearsal of the N > 1 bench
# modes; the driver runs the real 8-GPU RCCL line):  bash tools/gpu_r03_mr.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/mr}
mkdir -p "$out"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
run() {  # name port args...
  local name=$1 port=$2; shift 2
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --saturate 0 --probe= \
    --fresh-steps 0 "$@" > "$out/$name.json" 2> "$out/$name.err" || { tail -30 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$out/$name.json') if l.startswith('{')][-1]); print('$name', 'value=%.0f ms=%.2f' % (d['value'], d['ms_per_step']), d['result_decrypted'], d['config']['parallelism'][:60]); print('  per_rank', d['per_rank'])"
}
run weak_matches 29511 && run weak_matches_m4 29512 --matches 4 && run weak_starts 29513 --shard starts && \
run strong_closure 29514 --scaling strong && run strong_level 29515 --scaling strong --shard level
