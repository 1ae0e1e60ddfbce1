// Server-key generation on the device (the reference's
// ServerKey::new at src/regex/engine.rs:252 and gen_keys_radix at
// src/regex/ciphertext.rs:44).  Bit-identical to keys.cpp's gen_ksk +
// gen_bsk_torus followed by fft::bsk_to_fourier (and therefore to the oracle's
// keygen): the same ChaCha20 words (chacha.h) for every mask, exact mod-2^64
// sums for the bodies, the same host Box-Muller noise (uploaded), and the same
// butterfly sequence for the Fourier transform.
//
// Kernels (all integer / f64 add-and-multiply work, HBM-bound or LDS-bound):
//   k_gen_ksk      one wave per KSK row (kN * ks_level rows): masks from ChaCha
//                  blocks, <mask, s_small> reduced over the wave, + s_big[i] *
//                  2^(64 - B(j+1)) + noise
//   k_gen_bsk      one workgroup per GGSW row (w, r): masks A_j from ChaCha into
//                  LDS, body = sum_j A_j * S_j (negacyclic, binary S: one
//                  add/sub per set bit of S per coefficient) + noise, gadget m_w
//                  2^(64 - pbs_base_log) on coefficient 0 of component r
//   k_bsk_fourier  one workgroup per polynomial: fold, forward negacyclic FFT in
//                  LDS (fft.h butterflies, host twiddles), scale 2^-log2(M),
//                  written in the lane layouts of the blind-rotation kernels
//                  (E = 4; k = 2 also E = 8)
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "chacha.h"
#include "device.h"
#include "fft.h"
#include "geo.h"
#include "keys.h"

namespace fr {

#define KG_CHECK(x)                                                                          \
    do {                                                                                     \
        hipError_t _e = (x);                                                                 \
        if (_e != hipSuccess)                                                                \
            throw Error(FR_ERR_HIP, std::string("HIP error (keygen): ") + hipGetErrorString(_e)); \
    } while (0)

// u64 number 8*blk + q of a ChaCha stream: words (2q, 2q+1) of block blk
__device__ __forceinline__ uint64_t chacha_u64(const uint32_t* w, int q) {
    return (uint64_t)w[2 * q] | ((uint64_t)w[2 * q + 1] << 32);
}

// ksk[row][t], row = i * L + j; masks are u64 numbers row * n + t of STREAM_KSK_MASK
__global__ void __launch_bounds__(64) k_gen_ksk(uint64_t seed, int n, int L, int B, const uint64_t* __restrict__ s_small,
                                                const uint64_t* __restrict__ s_big, const int64_t* __restrict__ noise,
                                                uint64_t* __restrict__ ksk) {
    const int row = blockIdx.x, lane = threadIdx.x;
    const int i = row / L, j = row % L;
    const uint64_t first = (uint64_t)row * n, last = first + n;
    uint64_t* o = ksk + (size_t)row * (n + 1);
    uint64_t acc = 0;
    for (uint64_t b = (first >> 3) + lane; b <= ((last - 1) >> 3); b += 64) {
        uint32_t w[16];
        chacha_block(seed, STREAM_KSK_MASK, b, w);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t idx = b * 8 + q;
            if (idx >= first && idx < last) {
                const int t = (int)(idx - first);
                const uint64_t v = chacha_u64(w, q);
                o[t] = v;
                acc += v * s_small[t];
            }
        }
    }
    // wave sum mod 2^64 (order-free)
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) o[n] = acc + (s_big[i] << (64 - B * (j + 1))) + (uint64_t)noise[row];
}

// one GGSW row (w, r) of the torus BSK [w][r][c][coef]; 256 threads, N / 256
// coefficients per thread; LDS: the mask polynomial A_j (N u64)
template <int N>
__global__ void __launch_bounds__(256) k_gen_bsk(uint64_t seed, int k, const uint64_t* __restrict__ s_big,
                                                 const uint8_t* __restrict__ msg, const int32_t* __restrict__ noise,
                                                 uint64_t gadget, uint64_t* __restrict__ bsk) {
    constexpr int PER = N / 256;
    __shared__ uint64_t A[N];
    __shared__ uint32_t sbits[N / 32];
    const int kp1 = k + 1, tid = threadIdx.x;
    const int w = blockIdx.x / kp1, r = blockIdx.x % kp1;
    uint64_t* row = bsk + ((size_t)w * kp1 + r) * kp1 * N;
    uint64_t acc[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) acc[q] = 0;
    for (int j = 0; j < k; ++j) {
        const uint64_t base = (((uint64_t)w * kp1 + r) * k + j) * N;  // N % 8 == 0: whole ChaCha blocks
        for (int b = tid; b < N / 8; b += 256) {
            uint32_t wd[16];
            chacha_block(seed, STREAM_BSK_MASK, (base >> 3) + b, wd);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                uint64_t v = chacha_u64(wd, q);
                A[8 * b + q] = v;
                // the gadget lands on coefficient 0 of component r after the body used A
                if (j == r && b == 0 && q == 0 && msg[w]) v += gadget;
                row[(size_t)j * N + 8 * b + q] = v;
            }
        }
        const uint64_t* S = s_big + (size_t)j * N;
        for (int x = tid; x < N / 32; x += 256) {
            uint32_t m = 0;
            for (int y = 0; y < 32; ++y) m |= (uint32_t)(S[32 * x + y] & 1) << y;
            sbits[x] = m;
        }
        __syncthreads();
        // body += X^u A for every set bit u of S_j: coefficient t gets A[t - u]
        // (t >= u) or -A[t - u + N] (wrapped)
        for (int x = 0; x < N / 32; ++x) {
            uint32_t m = sbits[x];
            while (m) {
                const int u = 32 * x + __builtin_ctz(m);
                m &= m - 1;
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    const int t = tid + 256 * q;
                    const int d = t - u;
                    const uint64_t a = A[d >= 0 ? d : d + N];
                    acc[q] = d >= 0 ? acc[q] + a : acc[q] - a;
                }
            }
        }
        __syncthreads();
    }
    const int32_t* e = noise + ((size_t)w * kp1 + r) * N;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int t = tid + 256 * q;
        uint64_t v = acc[q] + (uint64_t)(int64_t)e[t];
        if (r == k && t == 0 && msg[w]) v += gadget;
        row[(size_t)k * N + t] = v;
    }
}

// element m of lane tl in the last-phase layout of lane geometry E (slot order, geo.h)
template <int M, int E>
__device__ __forceinline__ int lane_slot(int tl, int m) {
    constexpr int LOG = __builtin_ctz(M), e = __builtin_ctz(E), LAST = (LOG + e - 1) / e - 1;
    return geo_base(LOG, e, LAST, tl, fft_layout_variant(LOG, e)) + (m << geo_lo(LOG, e, LAST));
}
// fold + forward FFT + fourier_key_scale of one polynomial, written in the lane layouts of
// the E = 4, 8 and 16 kernels ([poly][m][lane], slot of (lane, m) per geo.h; a null
// output is skipped)
template <int N>
__global__ void __launch_bounds__(256) k_bsk_fourier(const uint64_t* __restrict__ bsk, const double2* __restrict__ tw,
                                                     double2* __restrict__ out4, double2* __restrict__ out8,
                                                     double2* __restrict__ out16) {
    constexpr int M = N / 2;
    constexpr int LOG = __builtin_ctz(M);
    __shared__ double2 z[M];
    const int tid = threadIdx.x;
    const size_t p = blockIdx.x;
    const uint64_t* a = bsk + p * N;
    for (int i = tid; i < M; i += 256) z[i] = make_double2((double)(int64_t)a[i], (double)(int64_t)a[i + M]);
    __syncthreads();
    for (int s = 0; s < LOG; ++s) {
        const int h = M >> (s + 1);
        for (int bi = tid; bi < M / 2; bi += 256) {
            const int b = bi / h, j = b * 2 * h + bi % h;
            const double2 c = tw[(1 << s) + b];
            double2 lo = z[j], hi = z[j + h];
            fft::fwd_bf(lo.x, lo.y, hi.x, hi.y, c.x, c.y);
            z[j] = lo;
            z[j + h] = hi;
        }
        __syncthreads();
    }
    const double scale = fft::fourier_key_scale(LOG);  // 1/M and the accumulator unit (fft.h), exact
    for (int idx = tid; idx < M; idx += 256) {
        if (out4) {
            const double2 v = z[lane_slot<M, 4>(idx % (M / 4), idx / (M / 4))];
            out4[p * M + idx] = make_double2(v.x * scale, v.y * scale);
        }
        if (out8) {
            const double2 v = z[lane_slot<M, 8>(idx % (M / 8), idx / (M / 8))];
            out8[p * M + idx] = make_double2(v.x * scale, v.y * scale);
        }
        if (out16) {
            const double2 v = z[lane_slot<M, 16>(idx % (M / 16), idx / (M / 16))];
            out16[p * M + idx] = make_double2(v.x * scale, v.y * scale);
        }
    }
}

// fresh LWE encryptions of block messages under the big key straight into
// arena slots (encrypt_str, src/regex/ciphertext.rs:32-40):
// one wave per block; masks are u64 numbers qb * kN + t of STREAM_ENC_MASK
// (kN % 8 == 0: whole ChaCha blocks), body = <mask, s_big> + m 2^59 + noise
__global__ void __launch_bounds__(64) k_encrypt_blocks(uint64_t seed, int big, const uint64_t* __restrict__ s_big,
                                                       const uint8_t* __restrict__ msgs,
                                                       const int64_t* __restrict__ noise, uint64_t first_block,
                                                       const int* __restrict__ slots, int stride,
                                                       uint64_t* __restrict__ arena) {
    const int q = blockIdx.x, lane = threadIdx.x;
    const uint64_t qb = first_block + q;
    uint64_t* o = arena + (size_t)slots[q] * stride;
    uint64_t acc = 0;
    for (int b = lane; b < big / 8; b += 64) {
        uint32_t w[16];
        chacha_block(seed, STREAM_ENC_MASK, qb * (uint64_t)(big / 8) + b, w);
#pragma unroll
        for (int x = 0; x < 8; ++x) {
            const uint64_t v = chacha_u64(w, x);
            o[8 * b + x] = v;
            acc += v * s_big[8 * b + x];
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) o[big] = acc + ((uint64_t)msgs[q] << DELTA_LOG) + (uint64_t)noise[q];
}

void Device::encrypt_to_slots(const ClientKey& ck, const uint8_t* msgs, size_t count, uint64_t seed,
                              uint64_t first_block, const int* slots) {
    if (!count) return;
    const int big = p_.big();
    if (big % 8) throw Error(FR_ERR_INVALID, "device encryption: kN must be a multiple of 8");
    if (ck.s_big.size() != (size_t)big) throw Error(FR_ERR_INVALID, "device encryption: key size");
    for (size_t i = 0; i < count; ++i)
        if (slots[i] < 0 || (size_t)slots[i] >= next_slot_) throw Error(FR_ERR_INVALID, "device encryption: slot");
    std::vector<int64_t> noise;
    enc_noise(p_, seed, first_block, count, noise);
    const hipStream_t s = (hipStream_t)stream_;
    uint64_t* d_sb = nullptr;
    uint8_t* d_m = nullptr;
    int64_t* d_n = nullptr;
    int* d_sl = nullptr;
    auto cleanup = [&] {
        (void)hipFree(d_sb);
        (void)hipFree(d_m);
        (void)hipFree(d_n);
        (void)hipFree(d_sl);
    };
    try {
        KG_CHECK(hipMalloc(&d_sb, 8 * (size_t)big));
        KG_CHECK(hipMalloc(&d_m, count));
        KG_CHECK(hipMalloc(&d_n, 8 * count));
        KG_CHECK(hipMalloc(&d_sl, 4 * count));
        KG_CHECK(hipMemcpyAsync(d_sb, ck.s_big.data(), 8 * (size_t)big, hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_m, msgs, count, hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_n, noise.data(), 8 * count, hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_sl, slots, 4 * count, hipMemcpyHostToDevice, s));
        k_encrypt_blocks<<<(unsigned)count, 64, 0, s>>>(seed, big, d_sb, d_m, d_n, first_block, d_sl, p_.slot_stride(),
                                                       d_arena_);
        KG_CHECK(hipGetLastError());
        KG_CHECK(hipStreamSynchronize(s));
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
}

void Device::gen_server_key(const ClientKey& ck, uint64_t seed) {
    if (p_.ring != FR_RING_FFT || !((p_.N == 2048 && p_.k == 1) || (p_.N == 1024 && p_.k == 2)))
        throw Error(FR_ERR_INVALID, "device keygen: FFT ring, (k, N) in {(1, 2048), (2, 1024)}");
    const int N = p_.N, M = N / 2, kp1 = p_.k + 1, n = p_.n, L = p_.ks_level;
    const size_t rows = (size_t)p_.big() * L, nw = p_.bsk_ggsw();
    const size_t bsk_polys = nw * kp1 * kp1;
    // every queued launch of every lane that reads the old keys has finished before they go
    KG_CHECK(hipDeviceSynchronize());
    // host: the noise draws and per-GGSW messages
    std::vector<int64_t> ksk_noise;
    std::vector<int32_t> bsk_noise;
    gen_ksk_noise(p_, seed, ksk_noise);
    gen_bsk_noise_torus(p_, seed, bsk_noise);
    const std::vector<uint8_t> msg = ggsw_messages(p_, ck);

    uint64_t *d_ss = nullptr, *d_sb = nullptr;
    int64_t* d_kn = nullptr;
    int32_t* d_bn = nullptr;
    uint8_t* d_msg = nullptr;
    auto cleanup = [&] {
        (void)hipFree(d_ss);
        (void)hipFree(d_sb);
        (void)hipFree(d_kn);
        (void)hipFree(d_bn);
        (void)hipFree(d_msg);
    };
    try {
        const hipStream_t s = (hipStream_t)stream_;
        KG_CHECK(hipMalloc(&d_ss, 8 * ck.s_small.size()));
        KG_CHECK(hipMalloc(&d_sb, 8 * ck.s_big.size()));
        KG_CHECK(hipMalloc(&d_kn, 8 * ksk_noise.size()));
        KG_CHECK(hipMalloc(&d_bn, 4 * bsk_noise.size()));
        KG_CHECK(hipMalloc(&d_msg, msg.size()));
        KG_CHECK(hipMemcpyAsync(d_ss, ck.s_small.data(), 8 * ck.s_small.size(), hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_sb, ck.s_big.data(), 8 * ck.s_big.size(), hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_kn, ksk_noise.data(), 8 * ksk_noise.size(), hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_bn, bsk_noise.data(), 4 * bsk_noise.size(), hipMemcpyHostToDevice, s));
        KG_CHECK(hipMemcpyAsync(d_msg, msg.data(), msg.size(), hipMemcpyHostToDevice, s));

        // KSK (torus) and its byte limbs
        (void)hipFree(d_ksk_);
        d_ksk_ = nullptr;
        KG_CHECK(hipMalloc(&d_ksk_, 8 * rows * (n + 1)));
        k_gen_ksk<<<(unsigned)rows, 64, 0, s>>>(seed, n, L, p_.ks_base_log, d_ss, d_sb, d_kn, d_ksk_);
        KG_CHECK(hipGetLastError());
        build_ksk_limbs();

        // torus BSK, kept for export
        (void)hipFree(d_tbsk_);
        d_tbsk_ = nullptr;
        KG_CHECK(hipMalloc(&d_tbsk_, 8 * p_.bsk_len()));
        const uint64_t gadget = 1ULL << (64 - p_.pbs_base_log);
        if (N == 2048) k_gen_bsk<2048><<<(unsigned)(nw * kp1), 256, 0, s>>>(seed, p_.k, d_sb, d_msg, d_bn, gadget, d_tbsk_);
        else k_gen_bsk<1024><<<(unsigned)(nw * kp1), 256, 0, s>>>(seed, p_.k, d_sb, d_msg, d_bn, gadget, d_tbsk_);
        KG_CHECK(hipGetLastError());

        // Fourier BSK in the lane layouts of the shapes in use (E = 4, and the throughput shape's)
        for (int E : {4, 8, 16}) {
            double*& dst = d_fbsk_[fbsk_index(E)];
            (void)hipFree(dst);
            dst = nullptr;
            if (fbsk_needed(E) && (E < 16 || p_.k == 1)) KG_CHECK(hipMalloc(&dst, 16 * bsk_polys * M));
        }
        double2 *o4 = (double2*)d_fbsk_[0], *o8 = (double2*)d_fbsk_[1], *o16 = (double2*)d_fbsk_[2];
        if (N == 2048)
            k_bsk_fourier<2048><<<(unsigned)bsk_polys, 256, 0, s>>>(d_tbsk_, (const double2*)d_ftw_, o4, o8, o16);
        else
            k_bsk_fourier<1024><<<(unsigned)bsk_polys, 256, 0, s>>>(d_tbsk_, (const double2*)d_ftw_, o4, o8, o16);
        KG_CHECK(hipGetLastError());
        KG_CHECK(hipStreamSynchronize(s));
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
}

void Device::download_server_key(uint64_t* ksk, size_t ksk_len, uint64_t* bsk, size_t bsk_len) {
    if (!d_ksk_ || !d_tbsk_) throw Error(FR_ERR_NO_KEY, "no device-generated server key");
    if (ksk) {
        if (ksk_len != (size_t)p_.big() * p_.ks_level * (p_.n + 1)) throw Error(FR_ERR_INVALID, "ksk size");
        KG_CHECK(hipMemcpy(ksk, d_ksk_, 8 * ksk_len, hipMemcpyDeviceToHost));
    }
    if (bsk) {
        if (bsk_len != p_.bsk_len()) throw Error(FR_ERR_INVALID, "bsk size");
        KG_CHECK(hipMemcpy(bsk, d_tbsk_, 8 * bsk_len, hipMemcpyDeviceToHost));
    }
}

}  // namespace fr
