// Microbenchmarks of the integer instruction rates the gate-bootstrap kernel
// depends on (gfx950): v_mad_u64_u32, 64-bit add, Goldilocks mul/butterfly.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "goldilocks.h"
using namespace fr;

template <int OP>
__global__ void __launch_bounds__(256) kern(uint64_t* out, uint64_t seed, int iters) {
    uint64_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = seed * (threadIdx.x + 1) * (i + 3) + blockIdx.x;
    const uint64_t z = seed | 0x123456789ULL;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) x[i] = (uint64_t)(uint32_t)x[i] * (uint32_t)z + x[i];  // v_mad_u64_u32
            if (OP == 1) x[i] = x[i] + z;                                       // 64-bit add
            if (OP == 2) x[i] = gl_mul(x[i], z);                                // Goldilocks mul
            if (OP == 3) { uint64_t t = gl_mul(z, x[i]); x[i] = gl_add(x[i], t) ^ gl_sub(x[i], t); }
            if (OP == 4) x[i] = (uint64_t)((uint32_t)x[i] * (uint32_t)z) + x[i];  // v_mul_lo_u32
        }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
double run(uint64_t* d, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    hipEventRecord(a);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double ops = (double)blocks * 256 * iters * 8;
    return ops / (ms * 1e-3);
}
int main() {
    uint64_t* d; hipMalloc(&d, 8ull * 256 * 8192);
    const char* names[] = {"mad_u64_u32", "add64", "gl_mul", "butterfly", "mul_lo_u32"};
    for (int blocks : {1024, 4096, 8192}) {
        double r[5];
        r[0] = run<0>(d, blocks, 4096); r[1] = run<1>(d, blocks, 4096); r[2] = run<2>(d, blocks, 1024);
        r[3] = run<3>(d, blocks, 1024); r[4] = run<4>(d, blocks, 4096);
        for (int i = 0; i < 5; ++i) printf("blocks=%d %-12s %8.2f G/s  (%.2f per CU-clock @2.4GHz)\n", blocks, names[i], r[i] / 1e9, r[i] / 256 / 2.4e9);
    }
    return 0;
}
