// Cost of the non-canonical Goldilocks ops (gl_device.h) vs the canonical ones.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "gl_device.h"
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
            if (OP == 5) { x[i] = gd::mul2(x[i], z); x[i+1] = gd::mul2(x[i+1], z); }
            if (OP == 6) gd::ct2(x[i], x[i+1], z);
            if (OP == 7) gd::gs2(x[i], x[i+1], z);
        }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void check(uint64_t* out) {
    // edge values around 0, P, 2^64 plus lane-derived pseudo-random ones
    const uint64_t edges[8] = {0, 1, P - 1, P, P + 1, ~0ULL, 0xFFFFFFFFULL, 0x100000000ULL};
    uint64_t s = 0x9E3779B97F4A7C15ULL * (threadIdx.x + 1);
    uint64_t err = 0;
    for (int it = 0; it < 4096; ++it) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        uint64_t a = (it & 7) == 0 ? edges[(it >> 3) & 7] : s;
        uint64_t b = (it & 15) == 1 ? edges[(it >> 4) & 7] : s * 0xD1B54A32D192ED03ULL;
        const uint64_t ac = a >= P ? a - P : a, bc = b >= P ? b - P : b;
        uint64_t m = gd::mul2(a, b);
        if (gd::canon(m) != gl_mul(ac, bc)) err = 1;
        if (gd::canon(gd::add_c2(a, bc)) != gl_add(ac, bc)) err = 2;
        if (gd::canon(gd::sub_c2(a, bc)) != gl_sub(ac, bc)) err = 3;
        uint64_t x = a, y = b, x2 = ac, y2 = bc;
        gd::ct2(x, y, bc);
        uint64_t t = gl_mul(bc, y2);
        if (gd::canon(x) != gl_add(x2, t) || gd::canon(y) != gl_sub(x2, t)) err = 4;
    }
    out[8 * threadIdx.x] = err;
}
template <int OP> double run(uint64_t* d, int blocks, int iters) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    (void)hipEventRecord(a); kern<OP><<<blocks, 256>>>(d, 7, iters); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    return (double)blocks * 256 * iters * ((OP >= 2 && OP != 5) ? 4 : 8) / (ms * 1e-3);
}
int main() {
    uint64_t* d; (void)hipMalloc(&d, 8ull * 256 * 8192);
    const char* names[] = {"gl_mul(canon)", "gd::mul(nc)", "bf canon", "gd::ct", "gd::gs", "gd::mul2", "gd::ct2", "gd::gs2"};
    double r[8] = {run<0>(d, 8192, 512), run<1>(d, 8192, 512), run<2>(d, 8192, 512), run<3>(d, 8192, 512), run<4>(d, 8192, 512),
                   run<5>(d, 8192, 512), run<6>(d, 8192, 512), run<7>(d, 8192, 512)};
    for (int i = 0; i < 8; ++i) printf("%-14s %8.2f G/s  %.2f per CU-clk  (~%.1f full-rate slots)\n", names[i], r[i] / 1e9, r[i] / 256 / 2.4e9, 128.0 / (r[i] / 256 / 2.4e9));
    // correctness: mul2/red2/add_c2/sub_c2 against the canonical host ops on edge + random values
    check<<<1, 256>>>(d);
    uint64_t h[256 * 8];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) if (h[8 * i]) { if (bad < 5) printf("MISMATCH lane %d code %llu\n", i, (unsigned long long)h[8 * i]); ++bad; }
    printf("variant-2 correctness: %s (%d bad lanes)\n", bad ? "FAIL" : "ok", bad);
    return 0;
}
