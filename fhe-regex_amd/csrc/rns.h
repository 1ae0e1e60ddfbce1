// The GLWE/GGSW ring of the blind rotation: Z_Q[X]/(X^N+1) with
// Q = p0 * p1, two 30-bit NTT primes, held in residue (RNS) form.
//
//   p0 = 998244353 = 119*2^23 + 1,  p1 = 1004535809 = 479*2^21 + 1
//   Q  = 1002772198720536577 (~2^59.8)
//
// Both primes are below 2^30, so NTT butterflies run Harvey-lazy in [0, 4p)
// with 32-bit adds, v_min_u32 reductions and Montgomery products (R = 2^32) —
// no carry flags, no 64-bit compares.  Data is kept in normal form; twiddles
// and the NTT-domain bootstrapping key are in Montgomery form.
//
// Everything that crosses the boundary stays on the 2^64 torus (tfhe-rs
// shortint): keyswitching, modulus switching, inputs and sample-extracted
// outputs.  The maps between the two worlds are exact integer functions,
// restated independently (with 128-bit arithmetic) by oracle/tfhe_oracle.c:
//   * decompose(x):  x = r0 + p0*k (k < p1), t = (k*round(2^61/p1) + 2^37) >> 38,
//                    digit = t (t < 2^22) or t - 2^23;  gadget G = round(Q / 2^23)
//   * to_torus(x):   sum_i round(2^64 * u_i / p_i) mod 2^64,
//                    u_i = x * (Q/p_i)^-1 mod p_i   (= round(x * 2^64 / Q) +- 1)
#pragma once
#include <cstdint>

#include "common.h"

namespace fr {
namespace rns {

constexpr uint32_t P0 = 998244353u, P1 = 1004535809u;
constexpr uint32_t PN0 = 998244351u, PN1 = 1004535807u;  // -p^-1 mod 2^32
constexpr uint32_t R2_0 = 932051910u, R2_1 = 542374313u;  // 2^64 mod p (to Montgomery form)
constexpr uint64_t Q = 1002772198720536577ULL;
constexpr uint64_t G = 119539761391ULL;          // round(Q / 2^23): gadget factor of the BSK
constexpr uint64_t H_Q = 15668315605008384ULL;   // round(Q / 64) = Delta/2 in Z_Q
constexpr uint64_t D_Q = 2 * H_Q;                // Delta in Z_Q
constexpr uint64_t A0 = 18479187002ULL, A1 = 18363450967ULL;  // floor(2^64 / p)
constexpr uint32_t B0 = 932051910u, B1 = 542374313u;          // 2^64 mod p
constexpr uint32_t CRT_CR = 334844587u;    // (p0^-1 mod p1) * 2^32 mod p1
constexpr uint32_t C0 = 332747959u;        // (Q/p0)^-1 = p1^-1 mod p0
constexpr uint32_t C1 = 669690699u;        // (Q/p1)^-1 = p0^-1 mod p1
constexpr uint32_t C0R = (uint32_t)(((uint64_t)C0 << 32) % P0);  // Montgomery forms
constexpr uint32_t C1R = (uint32_t)(((uint64_t)C1 << 32) % P1);
// Delta and Delta/2 residues (test-polynomial values), and Delta in Montgomery form
constexpr uint32_t DQ0 = (uint32_t)(D_Q % P0), DQ1 = (uint32_t)(D_Q % P1);
constexpr uint32_t HQ0 = (uint32_t)(H_Q % P0), HQ1 = (uint32_t)(H_Q % P1);
constexpr uint32_t DQR0 = (uint32_t)(((uint64_t)DQ0 << 32) % P0), DQR1 = (uint32_t)(((uint64_t)DQ1 << 32) % P1);
constexpr uint32_t GENERATOR = 3;          // of both multiplicative groups

// p = C * 2^K + 1 with K >= 16, so -p^-1 mod 2^32 = C * 2^K - 1 = p - 2
constexpr uint32_t PC0 = 119, PK0 = 23, PC1 = 479, PK1 = 21;
static_assert(P0 == PC0 * (1u << PK0) + 1 && P1 == PC1 * (1u << PK1) + 1, "prime shape");
static_assert(PN0 == P0 - 2 && PN1 == P1 - 2, "Montgomery constant");
FR_HD uint32_t prime(int i) { return i ? P1 : P0; }
FR_HD uint32_t pneg(int i) { return i ? PN1 : PN0; }
FR_HD uint64_t recip(int i) { return i ? A1 : A0; }

// ---- Montgomery arithmetic mod p (R = 2^32)
// a*b*R^-1 mod p, lazy result in [0, 2p) when a*b < 4p^2
FR_HD uint32_t mont_lazy(uint32_t a, uint32_t b, uint32_t p, uint32_t pn) {
    const uint64_t t = (uint64_t)a * b;
    const uint32_t m = (uint32_t)t * pn;
    return (uint32_t)((t + (uint64_t)m * p) >> 32);
}
FR_HD uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
// [0, 2p) -> [0, p) ;  [0, 4p) -> [0, 2p)
FR_HD uint32_t red1(uint32_t x, uint32_t p) { return umin(x, x - p); }
FR_HD uint32_t red2(uint32_t x, uint32_t p) { return umin(x, x - 2 * p); }
FR_HD uint32_t mont(uint32_t a, uint32_t b, uint32_t p, uint32_t pn) { return red1(mont_lazy(a, b, p, pn), p); }
FR_HD uint32_t addm(uint32_t a, uint32_t b, uint32_t p) { return red1(a + b, p); }
FR_HD uint32_t subm(uint32_t a, uint32_t b, uint32_t p) { const uint32_t d = a - b; return umin(d, d + p); }
FR_HD uint32_t negm(uint32_t a, uint32_t p) { return red1(p - a, p); }

// ---- 64-bit helpers
// floor(v * m / 2^64) for v < 2^64, m < 2^32
FR_HD uint64_t mulhi_32(uint64_t v, uint64_t m) {
    const uint64_t t = (v & 0xFFFFFFFFULL) * m;
    const uint64_t u = (v >> 32) * m + (t >> 32);
    return u >> 32;
}
// floor(w / p) for w < 2^62, with a = floor(2^64 / p) < 2^35 (one correction step)
FR_HD uint64_t div_p(uint64_t w, uint32_t p, uint64_t a) {
    const uint64_t a0 = a & 0xFFFFFFFFULL, a1 = a >> 32;
    // q_est = floor(w * a / 2^64) from 32-bit limbs
    const uint64_t w0 = w & 0xFFFFFFFFULL, w1 = w >> 32;
    const uint64_t ll = w0 * a0;
    const uint64_t mid = w0 * a1 + w1 * a0 + (ll >> 32);  // < 2^64 for w < 2^62, a < 2^35
    uint64_t q = w1 * a1 + (mid >> 32);
    const uint64_t r = w - q * p;
    if (r >= p) q += 1;
    return q;
}

// ---- the boundary maps
// x mod p for x < 2^62
FR_HD uint32_t reduce64(uint64_t x, int i) { return (uint32_t)(x - div_p(x, prime(i), recip(i)) * prime(i)); }
// CRT: residues (canonical) -> x in [0, Q)
FR_HD uint32_t crt_k(uint32_t r0, uint32_t r1);
FR_HD uint64_t crt(uint32_t r0, uint32_t r1) { return (uint64_t)r0 + (uint64_t)P0 * crt_k(r0, r1); }
// Signed gadget digit of x in Z_Q from its residues: with x = r0 + p0*k
// (k = (r1 - r0) * p0^-1 mod p1, exact), t = round-ish(k * 2^23 / p1) =
// (k * DIG_M + 2^37) >> 38 in [0, 2^23], recentred to [-2^22, 2^22).
// (x - digit * G) mod Q stays within 0.51 G.
constexpr uint32_t DIG_M = 2295431371u;  // round(2^61 / p1)
// (r1 - r0 + p1 in (0, 2p1): mont_lazy takes it unreduced)
FR_HD uint32_t crt_k(uint32_t r0, uint32_t r1) { return mont(r1 - r0 + P1, CRT_CR, P1, PN1); }
FR_HD int32_t digit_of_k(uint32_t k) {
    const uint32_t t = (uint32_t)(((uint64_t)k * DIG_M + (1ULL << 37)) >> 38);
    return t >= (1u << 22) ? (int32_t)t - (1 << 23) : (int32_t)t;
}
FR_HD int32_t decompose(uint32_t r0, uint32_t r1) { return digit_of_k(crt_k(r0, r1)); }
// Z_Q (residues, canonical) -> 2^64 torus
FR_HD uint64_t to_torus(uint32_t r0, uint32_t r1) {
    const uint32_t u0 = mont(r0, C0R, P0, PN0);  // r0 * C0 mod p0
    const uint32_t u1 = mont(r1, C1R, P1, PN1);
    const uint64_t t0 = A0 * u0 + div_p((uint64_t)B0 * u0 + (P0 >> 1), P0, A0);
    const uint64_t t1 = A1 * u1 + div_p((uint64_t)B1 * u1 + (P1 >> 1), P1, A1);
    return t0 + t1;
}

}  // namespace rns
}  // namespace fr
