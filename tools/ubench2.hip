// Cost of the non-canonical Goldilocks ops (gl_device.h) vs the canonical ones.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../fhe-regex_amd/csrc/gl_device.h"
using namespace fr;
template <int OP>
__global__ void __launch_bounds__(256) kern(uint64_t* out, uint64_t seed, int iters) {
    uint64_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = seed * (threadIdx.x + 1) * (i + 3) + blockIdx.x;
    const uint64_t z = seed | 0x123456789ULL;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            if (OP == 0) { x[i] = gl_mul(x[i], z); x[i+1] = gl_mul(x[i+1], z); }
            if (OP == 1) { x[i] = gd::mul(x[i], z); x[i+1] = gd::mul(x[i+1], z); }
            if (OP == 2) { uint64_t t = gl_mul(z, x[i+1]); uint64_t a = gl_add(x[i], t), b = gl_sub(x[i], t); x[i] = a; x[i+1] = b; }
            if (OP == 3) gd::ct(x[i], x[i+1], z);
            if (OP == 4) gd::gs(x[i], x[i+1], z);
        }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP> double run(uint64_t* d, int blocks, int iters) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    (void)hipEventRecord(a); kern<OP><<<blocks, 256>>>(d, 7, iters); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    return (double)blocks * 256 * iters * (OP >= 2 ? 4 : 8) / (ms * 1e-3);
}
int main() {
    uint64_t* d; (void)hipMalloc(&d, 8ull * 256 * 8192);
    const char* names[] = {"gl_mul(canon)", "gd::mul(nc)", "bf canon", "gd::ct", "gd::gs"};
    double r[5] = {run<0>(d, 8192, 512), run<1>(d, 8192, 512), run<2>(d, 8192, 512), run<3>(d, 8192, 512), run<4>(d, 8192, 512)};
    for (int i = 0; i < 5; ++i) printf("%-14s %8.2f G/s  %.2f per CU-clk  (~%.1f full-rate slots)\n", names[i], r[i] / 1e9, r[i] / 256 / 2.4e9, 128.0 / (r[i] / 256 / 2.4e9));
    // correctness spot check vs host gl_mul on one value
    return 0;
}
