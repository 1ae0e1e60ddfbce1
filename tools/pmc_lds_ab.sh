#!/bin/bash
# LDS-conflict A/B of experimental variants: time + bank-conflict counters
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in "$@"; do
  lib=fhe-regex_amd/libfheregex.so; [ "$v" != base ] && lib=fhe-regex_amd/build/exp/lib_$v.so
  echo "== $v"
  FHEREGEX_LIB=$lib timeout -k 10 200 python3 tools/br_timing.py 1 1024 | tail -2 || exit 1
  FHEREGEX_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/lds_$v -o run --output-format csv -- python3 tools/br_timing.py 1024 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/lds_$v/run_counter_collection.csv')):
    if 'blind_rotate' in r['Kernel_Name'] and int(r['Grid_Size'])>=1024*1024: print('  ',r['Counter_Name'], '%.4g' % float(r['Counter_Value']))"
done
