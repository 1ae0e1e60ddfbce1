// RNS (two 31-bit primes, Montgomery) butterfly cost vs Goldilocks, gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "gl_device.h"
using namespace fr;
struct MP { uint32_t p, pinv_neg; };  // -p^-1 mod 2^32
__device__ __forceinline__ uint32_t mont(uint32_t a, uint32_t b, uint32_t p, uint32_t pn) {
    uint64_t t = (uint64_t)a * b;
    uint32_t m = (uint32_t)t * pn;
    uint64_t u = t + (uint64_t)m * p;      // < 2^64, low 32 bits zero
    uint32_t r = (uint32_t)(u >> 32);      // < 2p
    return min(r, r - p);
}
__device__ __forceinline__ uint32_t addm(uint32_t a, uint32_t b, uint32_t p) { uint32_t s = a + b; return min(s, s - p); }
__device__ __forceinline__ uint32_t subm(uint32_t a, uint32_t b, uint32_t p) { uint32_t d = a - b; return min(d, d + p); }
__device__ __forceinline__ void ct_rns(uint32_t& x, uint32_t& y, uint32_t w, uint32_t p, uint32_t pn) {
    uint32_t t = mont(w, y, p, pn); y = subm(x, t, p); x = addm(x, t, p);
}
// m via v_mad_u64_u32 (half rate) instead of v_mul_lo_u32 (quarter rate)
__device__ __forceinline__ uint32_t mont2(uint32_t a, uint32_t b, uint32_t p, uint32_t pn) {
    uint64_t t = (uint64_t)a * b;
    uint32_t m = (uint32_t)(uint64_t)((uint64_t)(uint32_t)t * pn);
    uint64_t u = t + (uint64_t)m * p;
    uint32_t r = (uint32_t)(u >> 32);
    return min(r, r - p);
}
__device__ __forceinline__ void ct_rns2(uint32_t& x, uint32_t& y, uint32_t w, uint32_t p, uint32_t pn) {
    uint32_t t = mont2(w, y, p, pn); y = subm(x, t, p); x = addm(x, t, p);
}
// Harvey lazy CT butterfly, p < 2^30: x,y in [0,4p) -> [0,4p)
__device__ __forceinline__ void ct_lazy(uint32_t& x, uint32_t& y, uint32_t w, uint32_t p, uint32_t pn) {
    x = min(x, x - 2 * p);                    // [0, 2p)
    uint64_t t64 = (uint64_t)w * y;
    uint32_t m = (uint32_t)t64 * pn;
    uint32_t t = (uint32_t)((t64 + (uint64_t)m * p) >> 32);  // [0, 2p)
    y = x - t + 2 * p;
    x = x + t;
}
template <int OP>
__global__ void __launch_bounds__(256) kern(uint64_t* out, uint64_t seed, int iters) {
    const uint32_t P1 = 2013265921u, P1N = 2013265919u, P2 = 2130706433u, P2N = 2130706431u;
    const uint32_t Q1 = 998244353u, Q1N = 998244351u, Q2 = 1004535809u, Q2N = 1004535807u;
    uint32_t x[8], y[8];
    uint64_t X[8];
    for (int i = 0; i < 8; ++i) { X[i] = seed * (threadIdx.x + 1) * (i + 3) + blockIdx.x; x[i] = (uint32_t)X[i] % P1; y[i] = (uint32_t)(X[i] >> 32) % P2; }
    const uint64_t z = seed | 0x123456789ULL;
    const uint32_t w1 = (uint32_t)z % P1, w2 = (uint32_t)(z >> 32) % P2;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            if (OP == 0) gd::ct(X[i], X[i + 1], z);
            if (OP == 1) { ct_rns(x[i], x[i + 1], w1, P1, P1N); ct_rns(y[i], y[i + 1], w2, P2, P2N); }
            if (OP == 2) { ct_rns2(x[i], x[i + 1], w1, P1, P1N); ct_rns2(y[i], y[i + 1], w2, P2, P2N); }
            if (OP == 3) { ct_lazy(x[i], x[i + 1], w1, Q1, Q1N); ct_lazy(y[i], y[i + 1], w2, Q2, Q2N); }
        }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= X[i] ^ x[i] ^ ((uint64_t)y[i] << 32);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP> double run(uint64_t* d, int blocks, int iters) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    (void)hipEventRecord(a); kern<OP><<<blocks, 256>>>(d, 7, iters); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    return (double)blocks * 256 * iters * 4 / (ms * 1e-3);
}
int main() {
    uint64_t* d; (void)hipMalloc(&d, 8ull * 256 * 8192);
    double r[4] = {run<0>(d, 8192, 512), run<1>(d, 8192, 512), run<2>(d, 8192, 512), run<3>(d, 8192, 512)};
    const char* nm[4] = {"goldilocks ct", "RNS 2x31 ct", "RNS 2x31 ct (mad m)", "RNS 2x30 Harvey lazy"};
    for (int i = 0; i < 4; ++i) printf("%-22s %8.2f G/s  (~%.1f slots)\n", nm[i], r[i] / 1e9, 128.0 / (r[i] / 256 / 2.4e9));
    return 0;
}
