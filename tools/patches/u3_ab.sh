set -o pipefail
out=gpurun_out/r05b; mkdir -p $out
timeout -k 10 200 ./tools/ubench_keystream > $out/ubench_keystream.log 2>&1 || { echo ubench failed; tail $out/ubench_keystream.log; exit 1; }
for r in 1 2; do
for v in "FR_U3=0" "FR_U3=1 FR_U3_TIMING=1 FR_U3_MAX=256"; do
  echo "== $v" >> $out/u3_lat.log
  env $v timeout -k 10 200 python tools/lat_probe.py 5 1 16 254 >> $out/u3_lat.log 2>&1 || { echo lat failed; tail $out/u3_lat.log; exit 1; }
done; done
for r in 1 2; do
for v in "FR_U3=0" "FR_U3=1 FR_U3_TIMING=1 FR_U3_MAX=16" "FR_U3=1 FR_U3_TIMING=1 FR_U3_MAX=256"; do
  echo "== $v" >> $out/u3_match.log
  env $v timeout -k 10 200 python tools/match_ab.py 7 >> $out/u3_match.log 2>&1 || { echo match failed; tail $out/u3_match.log; exit 1; }
done; done
cat $out/u3_lat.log $out/u3_match.log
