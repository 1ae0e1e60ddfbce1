set -o pipefail
out=gpurun_out/r04f; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dual_shape or match_words" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 700 bash tools/ab_env_r04.sh 3 - FR_FFT_DUAL=1 > $out/ab.log 2>&1 || { tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
