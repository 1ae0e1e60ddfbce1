set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/ab_bench.sh "FR_AB=new" "FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_noperm.so" || exit 1
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_timing.so timeout -k 10 120 python3 tools/br_timing.py 1 256 512
