// Shared definitions for the fheregex product library (host + device).
#pragma once
#include <cstdint>
#include <cstddef>
#include <string>
#include <stdexcept>

#include "fheregex.h"

#if defined(__HIPCC__)
#define FR_HD __host__ __device__ __forceinline__
#define FR_UNROLL _Pragma("unroll")
#else
#define FR_HD inline
#define FR_UNROLL
#endif

namespace fr {

// Encoding scale of a 16-value message with one padding bit (tfhe-rs shortint
// PARAM_MESSAGE_2_CARRY_2): Delta = 2^63 / 16 = 2^59 on the 2^64 torus.  The
// blind-rotation ring and its constants live in rns.h.
constexpr int DELTA_LOG = 59;

// Keyswitch signed decomposition: top B*L bits of a (rounded), digits in [-2^(B-1), 2^(B-1)),
// most significant level first (dig[0] has weight 2^(64-B)).
template <int B, int L>
FR_HD void ks_decompose(uint64_t a, int32_t* dig) {
    constexpr int bits = B * L;
    uint64_t c = (a >> (64 - bits)) + ((a >> (64 - bits - 1)) & 1);
    c &= (bits >= 64) ? ~0ULL : ((1ULL << bits) - 1);
FR_UNROLL
    for (int j = L - 1; j >= 0; --j) {
        uint64_t d = c & ((1ULL << B) - 1);
        c >>= B;
        if (d >= (1ULL << (B - 1))) {
            dig[j] = (int32_t)d - (1 << B);
            c += 1;
        } else {
            dig[j] = (int32_t)d;
        }
    }
}

FR_HD uint32_t mod_switch(uint64_t a, int log2N2) {
    return (uint32_t)((((a >> (64 - log2N2 - 1)) + 1) >> 1) & ((1ULL << log2N2) - 1));
}

// ---------------------------------------------------------------- errors
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
void set_last_error(const std::string& msg);

// ---------------------------------------------------------------- params
struct Params {
    int k = 1, N = 2048, n = 742;
    int ks_base_log = 3, ks_level = 5;
    int pbs_base_log = 23, pbs_level = 1;
    int ring = FR_RING_FFT;  // blind-rotation ring (fheregex.h)
    double lwe_sigma = 7.069849454709433e-06;
    double glwe_sigma = 2.9403601535432533e-16;
    int big() const { return k * N; }
    int lwe_len() const { return k * N + 1; }
    // device slot stride (u64) of a big LWE, padded to 64 B
    int slot_stride() const { return (lwe_len() + 7) & ~7; }
    int ks_stride() const { return (n + 1 + 7) & ~7; }
    int log2N() const { int l = 0; while ((1 << l) < N) ++l; return l; }
    // bootstrapping-key unrolling: LWE coefficients in pairs (3 GGSWs per pair:
    // s_i s_j, s_i(1-s_j), (1-s_i)s_j) for k = 1 and on the FFT ring; the RNS
    // ring at k > 1 keeps one GGSW per coefficient
    int bsk_unroll() const { return (k == 1 || ring == FR_RING_FFT) ? 2 : 1; }
    size_t bsk_ggsw() const { return bsk_unroll() == 2 ? 3 * (size_t)((n + 1) / 2) : (size_t)n; }
    size_t bsk_len() const { return bsk_ggsw() * (size_t)(k + 1) * (k + 1) * N; }
};
Params params_from_c(const fr_params* p);
void validate_params(const Params& p);

}  // namespace fr
