# FR_MAC_EARLY=1 A/B (latency shape) and its bit-exactness through the variant library
set -o pipefail
mkdir -p gpurun_out/r06i
SIZES="1 16 254" timeout -k 10 600 bash tools/ab_libs.sh 3 fhe-regex_amd/build/exp/lib_base.so fhe-regex_amd/build/exp/lib_macearly.so > gpurun_out/r06i/ab_macearly.log 2>&1 &&
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_macearly.so timeout -k 10 600 python -u -m pytest tests/test_fft.py tests/test_gpu.py tests/test_exact_br.py -m gpu -x -q --timeout 200 --timeout-method thread -k "blind_rotate or match_words_abc_64 or one_step or reference_vectors or pair_shape or config4_the" > gpurun_out/r06i/tests_macearly.log 2>&1
tail -3 gpurun_out/r06i/tests_macearly.log; cat gpurun_out/r06i/ab_macearly.log
