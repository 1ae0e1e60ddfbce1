#!/bin/bash
# Energy per bootstrap of the blind-rotation launches, and of timing-only variants that drop one
# part of the step (wrong results; timing and energy only):
#   nobsk  -DFR_FFT_NOBSK   no Fourier-key loads (the key stream from L2/HBM)
#   noxchg -DFR_FFT_NOXCHG  no LDS exchanges in the transforms
#   nomacx -DFR_FFT_NOMACX  no MAC exchange (and its barrier)
#   nopsi  -DFR_FFT_NOPSI   no monomial-table lookups
# built beforehand by tools/build_variant.sh NAME FLAGS; two interleaved rounds on one box.
# Output: gpurun_out/r06k/var_NAME_I/power.json (tools/power_probe.py)
set -o pipefail
out=gpurun_out/r06k
mkdir -p $out
for i in 1 2; do
  for v in base nobsk noxchg nomacx nopsi; do
    echo "== $v round $i"
    FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_$v.so timeout -k 10 120 python3 -u tools/power_probe.py $out/var_${v}_$i \
      --counts 254,512,2048 --no-match --idle 0.5 > $out/var_${v}_$i.log 2>&1 || { echo "FAILED $v $i"; tail -5 $out/var_${v}_$i.log; exit 1; }
    grep '"phase": "launch' $out/var_${v}_$i.log
  done
done
echo done
