// Checks the lane maps of v_mfma_i32_32x32x32_i8 on gfx950 with exact integers:
// A fragment: lane l holds A[l&31][16*(l>>5) + j], j < 16 (16 int8 = 4 VGPRs)
// B fragment: lane l holds B[16*(l>>5) + j][l&31]
// C/D: reg i of lane l is D[(i&3) + 8*(i>>2) + 4*(l>>5)][l&31]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const int8_t* A, const int8_t* B, int* D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; ++j) { a[j] = A[r * 32 + 16 * h + j]; b[j] = B[(16 * h + j) * 32 + r]; }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}
int main() {
    int8_t hA[1024], hB[1024];
    int ref[1024], got[1024];
    srand(7);
    for (int i = 0; i < 1024; ++i) { hA[i] = (int8_t)(rand() % 256 - 128); hB[i] = (int8_t)(rand() % 256 - 128); }
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int s = 0;
            for (int t = 0; t < 32; ++t) s += hA[i * 32 + t] * hB[t * 32 + j];
            ref[i * 32 + j] = s;
        }
    int8_t *dA, *dB; int* dD;
    (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dD, 4096);
    (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dD);
    (void)hipMemcpy(got, dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += got[i] != ref[i];
    printf("mfma_i32_32x32x32_i8 lane map: %s (%d mismatches)\n", bad ? "MISMATCH" : "ok", bad);
    return bad != 0;
}
