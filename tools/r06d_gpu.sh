# latency of small launches in the other k = 1 shapes (dual: 4 waves, both polynomials per lane;
# pair: two bootstraps per 8-wave workgroup) against the latency shape
set -o pipefail
mkdir -p gpurun_out/r06d
for r in 1 2; do
  timeout -k 10 120 python3 tools/lat_probe.py 7 1 16 254 > gpurun_out/r06d/lat_$r.log 2>&1 &&
  FR_FFT_SMALL_BATCH=0 FR_FFT_DUAL=1 timeout -k 10 120 python3 tools/lat_probe.py 7 1 16 254 > gpurun_out/r06d/dual_$r.log 2>&1 &&
  FR_FFT_SMALL_BATCH=0 timeout -k 10 120 python3 tools/lat_probe.py 7 1 16 254 > gpurun_out/r06d/pair_$r.log 2>&1 || exit 1
done
cat gpurun_out/r06d/*.log
