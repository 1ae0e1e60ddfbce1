#!/bin/bash
# PMC passes over tools/br_timing.py (one gate batch, default 1024) for the BR kernel:
#   tools/pmc_br.sh [outdir] [batch]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/pmc_br}; batch=${2:-1024}; mkdir -p "$out"; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" -d "$out/$name" -o run --output-format csv -- python3 tools/br_timing.py $batch > "$out/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }; }
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_LDS
run b SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
run c SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_BRANCH
echo ok
