#!/bin/bash
# parity + A/B bench + LDS PMC pass of the latency shape (current library)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_lat
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab_bench.sh "FR_AB=${1:-cur}" || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc_lat/cur -o run --output-format csv -- python3 tools/br_timing.py 256 > gpurun_out/pmc_lat/cur.log 2>&1 || exit 1
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_timing.so timeout -k 10 120 python3 tools/br_timing.py 1 512
