#!/bin/bash
# PMC passes over tools/ks_probe.py (keyswitch of 512 gates) for the keyswitch kernels:
#   tools/pmc_ks.sh [outdir]
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/pmc_ks}; mkdir -p "$out"; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d "$out/$name" -o run --output-format csv -- python3 tools/ks_probe.py 3 512 > "$out/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }; }
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run b SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_COUNT
run c TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
run d FETCH_SIZE
run e TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum
echo ok
