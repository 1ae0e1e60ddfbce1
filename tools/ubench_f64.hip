// Microbenchmarks of the f64 instruction rates an FFT-based blind rotation
// depends on (gfx950): v_fma_f64, v_add_f64, v_mul_f64, a radix-2 complex
// butterfly, against v_fma_f32 / v_add_u32 and the RNS Montgomery product.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_f64.hip -o tools/ubench_f64
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int OP>
__global__ void __launch_bounds__(256) kern(double* out, double seed, int iters) {
    double x[8], y[8];
    for (int i = 0; i < 8; ++i) {
        x[i] = seed * (threadIdx.x + 1) * (i + 3) + blockIdx.x;
        y[i] = seed * (i + 1);
    }
    const double wr = 0.70710678118654752, wi = -0.70710678118654752;
    float xf[8];
    uint32_t xu[8];
    for (int i = 0; i < 8; ++i) {
        xf[i] = (float)x[i];
        xu[i] = (uint32_t)(threadIdx.x * 77 + i);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) x[i] = __builtin_fma(x[i], wr, y[i]);  // v_fma_f64
            if (OP == 1) x[i] = x[i] + y[i];                    // v_add_f64
            if (OP == 2) x[i] = x[i] * wr;                      // v_mul_f64
            if (OP == 3 && i < 4) {                             // complex butterfly (x, y) pairs
                const double tr = __builtin_fma(y[2 * i], wr, -y[2 * i + 1] * wi);
                const double ti = __builtin_fma(y[2 * i], wi, y[2 * i + 1] * wr);
                const double ar = x[2 * i], ai = x[2 * i + 1];
                x[2 * i] = ar + tr;
                x[2 * i + 1] = ai + ti;
                y[2 * i] = ar - tr;
                y[2 * i + 1] = ai - ti;
            }
            if (OP == 4) xf[i] = __builtin_fmaf(xf[i], (float)wr, (float)wi);  // v_fma_f32
            if (OP == 5) xu[i] = xu[i] + (uint32_t)it;                          // v_add_u32
            if (OP == 6) {  // f64 -> i64 bits -> wrap (the backward torus conversion)
                const double v = x[i] * 1.5;
                x[i] = (double)(int64_t)__builtin_rint(v * 0x1p-40);
            }
        }
    }
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i] + y[i] + xf[i] + xu[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
double run(double* d, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    kern<OP><<<blocks, 256>>>(d, 1.000001, iters);
    hipEventRecord(a);
    kern<OP><<<blocks, 256>>>(d, 1.000001, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double per = OP == 3 ? 4 : 8;  // butterflies / ops per iteration
    return (double)blocks * 256 * iters * per / (ms * 1e-3);
}
int main() {
    double* d;
    hipMalloc(&d, 8ull * 256 * 8192);
    const char* names[] = {"fma_f64", "add_f64", "mul_f64", "cbutterfly", "fma_f32", "add_u32", "f64_to_i64"};
    for (int blocks : {2048, 8192}) {
        double r[7];
        r[0] = run<0>(d, blocks, 2048);
        r[1] = run<1>(d, blocks, 2048);
        r[2] = run<2>(d, blocks, 2048);
        r[3] = run<3>(d, blocks, 2048);
        r[4] = run<4>(d, blocks, 2048);
        r[5] = run<5>(d, blocks, 2048);
        r[6] = run<6>(d, blocks, 512);
        for (int i = 0; i < 7; ++i)
            printf("blocks=%d %-12s %9.2f G/s  (%.2f per CU-clock @2.4GHz)\n", blocks, names[i], r[i] / 1e9,
                   r[i] / 256 / 2.4e9);
    }
    return 0;
}
