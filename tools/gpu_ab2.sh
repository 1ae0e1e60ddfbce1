#!/bin/bash
# A/B of the DPP exchange variant + an LDS PMC pass of the latency shape.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/ab_bench.sh "FR_AB=new" "FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_dpp.so" || exit 1
mkdir -p gpurun_out/pmc_lat
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc_lat/def -o run --output-format csv -- python3 tools/br_timing.py 256 > gpurun_out/pmc_lat/def.log 2>&1 || exit 1
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_dpp.so timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc_lat/dpp -o run --output-format csv -- python3 tools/br_timing.py 256 > gpurun_out/pmc_lat/dpp.log 2>&1 || exit 1
echo done
