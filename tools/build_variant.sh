#!/bin/bash
# Build an experimental variant of libfheregex.so with extra -D flags:
#   tools/build_variant.sh NAME [-DFOO=1 ...]  ->  fhe-regex_amd/build/exp/lib_NAME.so
# (select it at run time with FHEREGEX_LIB=...)
set -e
cd "$(dirname "$0")/../fhe-regex_amd"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p build/exp
# the Makefile's SCHED for every TU (override with SCHED=...)
SCHED=${SCHED--mllvm --amdgpu-use-amdgpu-trackers}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc $SCHED "$@" -c csrc/device.hip -o build/exp/device_$name.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc $SCHED "$@" -c csrc/fft_br.hip -o build/exp/fft_br_$name.o
# the pair shape's translation unit under its scheduler (Makefile PAIR_SCHED; override with PAIR_SCHED=...)
PAIR_SCHED=${PAIR_SCHED--mllvm --amdgpu-sched-strategy=max-ilp}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc $SCHED $PAIR_SCHED "$@" -c csrc/fft_br_pair.hip -o build/exp/fft_br_pair_$name.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/exp/lib_$name.so build/keys.o build/fft.o build/regex.o build/merged.o build/lower.o build/capi.o build/keygen.o build/exp/device_$name.o build/exp/fft_br_$name.o build/exp/fft_br_pair_$name.o -lpthread
echo "built fhe-regex_amd/build/exp/lib_$name.so"
