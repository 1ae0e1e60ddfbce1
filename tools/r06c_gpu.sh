set -o pipefail
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
SIZES="1 16 254 512 2048" timeout -k 10 700 bash tools/ab_libs.sh 3 fhe-regex_amd/build/exp/lib_base.so fhe-regex_amd/build/exp/lib_prio1.so fhe-regex_amd/build/exp/lib_prio1lat.so > gpurun_out/r06c/ab_prio.log 2>&1 &&
FHEREGEX_LIB=fhe-regex_amd/build/exp/lib_timing.so timeout -k 10 120 python3 tools/br_timing.py 1 16 254 > gpurun_out/r06c/seg_timing.log 2>&1 &&
timeout -k 10 600 bash tools/pmc_br.sh gpurun_out/r06c/pmc_lat1 1 > gpurun_out/r06c/pmc.log 2>&1
