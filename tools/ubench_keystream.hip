// Key-stream rate of the latency-shape geometry (the test before
// building key unrolling by three): one 512-lane workgroup per CU reads a Fourier key
// laid out as the blind rotation reads it -- per step G groups, each lane 8 x 16 B per
// group (one wave instruction = 1 KB contiguous) -- through a ring of D groups held in
// registers, with W dependent f64 FMAs of "MAC work" per consumed group.
//   U = 2: 371 steps x 3 groups x 64 KB = 71 MB;  U = 3: 248 steps x 7 groups = 111 MB.
// Reported: GB/s per workgroup (bytes one workgroup streams / kernel time) for 1, 16 and
// 254 workgroups (16 / 254 read the same key, as bootstraps of one launch do).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_keystream tools/ubench_keystream.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

constexpr int LANES = 512;
constexpr int PER_LANE = 8;                                   // 16-byte loads per lane per group
constexpr size_t GROUP_BYTES = (size_t)LANES * PER_LANE * 16;  // 64 KB

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
struct Grp {
    v4u v[PER_LANE];
};

// one group's loads: raw buffer loads as the product's key loads (resource in SGPRs, the
// group's byte offset uniform in soffset, one lane offset VGPR): 8 x dwordx4 per lane
__device__ __forceinline__ void load_grp(Grp& g, __amdgpu_buffer_rsrc_t r, int lane_off, int grp) {
    const int soff = __builtin_amdgcn_readfirstlane(grp) * (int)GROUP_BYTES;
#pragma unroll
    for (int i = 0; i < PER_LANE; ++i)
        g.v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, lane_off + i * LANES * 16, soff, 0);
}
template <int W>
__device__ __forceinline__ void consume(const Grp& g, double& acc) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < PER_LANE; ++i)
        s += __hiloint2double((int)g.v[i].y, g.v[i].x) + __hiloint2double((int)g.v[i].w, g.v[i].z);
    // one serial chain through acc (at least one fma): the compiler cannot move a group's
    // consumption past the next group's loads
#pragma unroll
    for (int w = 0; w < (W > 0 ? W : 1); ++w) acc = fma(acc, 0.999999, s);
}

template <int D, int W>
__global__ void __launch_bounds__(LANES) k_stream(const uint4* __restrict__ key, int groups, double* out) {
    extern __shared__ char lds_pad[];  // dynamic LDS: one workgroup per CU
    const int tl = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)key, 0, 0x7fffffff, 0x00020000);
    const int lane_off = tl * 16;
    Grp g[D];
    double acc = (double)tl;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        load_grp(g[d], r, lane_off, d);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int g0 = 0; g0 < groups; g0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            // the ring's order is fixed (sched barriers): consuming group d waits for its
            // own loads only, the other D - 1 groups stay in flight
            consume<W>(g[d], acc);
            __builtin_amdgcn_sched_barrier(0);
            const int nxt = g0 + D + d;
            load_grp(g[d], r, lane_off, nxt < groups ? nxt : 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc == 1234.5) out[blockIdx.x * LANES + tl] = acc + lds_pad[tl];
}

template <int D, int W>
int run(const uint4* key, int groups, int wgs, double* out, float* best) {
    const size_t lds = 96 * 1024;
    CK(hipFuncSetAttribute((const void*)k_stream<D, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    *best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_stream<D, W>), dim3(wgs), dim3(LANES), lds, 0, key, groups, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < *best) *best = ms;  // rep 0: warm-up
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

template <int D, int W>
int row(const uint4* key, double* out, const char* what) {
    const int steps_u[2] = {371, 248}, gps[2] = {3, 7};
    for (int u = 0; u < 2; ++u) {
        const int groups = steps_u[u] * gps[u];
        const double mb = groups * (double)GROUP_BYTES / 1e6;
        for (int wgs : {1, 16, 254}) {
            float ms;
            if (run<D, W>(key, groups, wgs, out, &ms)) return 1;
            printf("U=%d D=%d W=%3d %-22s wgs=%3d  %7.1f MB  %8.3f ms  %7.1f GB/s per WG  %5.2f us per step\n", u + 2, D,
                   W, what, wgs, mb, ms, mb / ms, 1e3 * ms / steps_u[u]);
            fflush(stdout);
        }
    }
    return 0;
}

int main() {
    const size_t bytes = (size_t)248 * 7 * GROUP_BYTES;  // the U = 3 key, 113.8 MB
    uint4* key;
    double* out;
    CK(hipMalloc(&key, bytes));
    CK(hipMalloc(&out, (size_t)256 * LANES * sizeof(double)));
    CK(hipMemset(key, 0x3f, bytes));
    int rc = 0;
    rc |= row<1, 0>(key, out, "ring 1, 1 fma/group");
    rc |= row<2, 0>(key, out, "ring 2, 1 fma/group");
    rc |= row<3, 0>(key, out, "ring 3, 1 fma/group");
    rc |= row<4, 0>(key, out, "ring 4, 1 fma/group");
    rc |= row<3, 48>(key, out, "ring 3, 48 fma/group");
    rc |= row<4, 48>(key, out, "ring 4, 48 fma/group");
    rc |= row<3, 96>(key, out, "ring 3, 96 fma/group");
    CK(hipFree(key));
    CK(hipFree(out));
    return rc;
}
