#!/bin/bash
# On the GPU box: rocprofv3 kernel-trace stats and separate PMC passes (HBM
# bytes; SQ issue/stall buckets and VALU count; LDS + GRBM cycles) of the
# default bench, summarised by tools/pmc_summary.py into OUTDIR/pmc_summary.json.
#   bash tools/profile.sh OUTDIR [extra bench args]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/prof}
shift
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --cpu-sample 0 --probe= --fresh-steps 0 --faithful-steps 0 --faithful-tree-steps 0 --inflight 0 --lanes 0 $*"
step() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?"; exit 1; }; }
step 400 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 $B > "$out/trace.log" 2>&1
step 400 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_fetch" -o run --output-format csv -- python3 $B > "$out/pmc_fetch.log" 2>&1
step 400 rocprofv3 --pmc WRITE_SIZE -d "$out/pmc_write" -o run --output-format csv -- python3 $B > "$out/pmc_write.log" 2>&1
step 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_LDS -d "$out/pmc_sq" -o run --output-format csv -- python3 $B > "$out/pmc_sq.log" 2>&1
step 400 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d "$out/pmc_lds" -o run --output-format csv -- python3 $B > "$out/pmc_lds.log" 2>&1
k=1; case " $* " in *k2n1024*) k=2 ;; esac
python3 tools/pmc_summary.py "$out" "$out/pmc_summary.json" "$k"
echo done
