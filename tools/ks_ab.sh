#!/bin/bash
# keyswitch split/tile A/B: kernel-trace stats of the default bench per setting
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in "FR_KS_MC=1" "FR_KS_MC=2" "FR_KS_MC=2 FR_KS_TILES=8192" "FR_KS_MR4_MIN=100000"; do
  d=gpurun_out/ks_ab/$(echo $v | tr ' =' '__')
  mkdir -p $d
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > $d/log 2>&1 || { echo "fail $v"; exit 1; }
  echo "== $v"
  python3 - "$d" <<'PY'
import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'k_ks' in n:
        agg[(n.split('(')[0][-22:], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(agg.items()):
    print(k, len(v), 'avg %.1f us' % (sum(v) / len(v)))
PY
done
