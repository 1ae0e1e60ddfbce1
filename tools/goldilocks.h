// Goldilocks scalar arithmetic of the first (round-1) ring, kept for the
// microbenchmarks in tools/ only; the product uses rns.h.
#pragma once
#include "../fhe-regex_amd/csrc/common.h"
namespace fr {
// Goldilocks prime: the GLWE/GGSW ring is Z_p[X]/(X^N+1) (exact integer NTT;
// 2^32-th roots of unity exist, 2^64 = 2^32 - 1 and 2^96 = -1 mod p).
constexpr uint64_t P = 0xFFFFFFFF00000001ULL;
constexpr uint64_t EPS = 0xFFFFFFFFULL;  // 2^64 - P
// PBS gadget for base 2^23, one level: g = floor(P / 2^23); 2^23 * g = P - 1.
constexpr uint64_t PBS_G = (1ULL << 41) - (1ULL << 9);
// Encoding scale of a 16-value message with one padding bit (tfhe-rs shortint
// PARAM_MESSAGE_2_CARRY_2): Delta = 2^63 / 16 = 2^59 on the 2^64 torus, and
// round(2^59 * P / 2^64) = 2^59 - 2^27 in Z_p.
constexpr uint64_t DELTA_P = (1ULL << 59) - (1ULL << 27);

FR_HD uint64_t gl_add(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    uint64_t t = s + EPS;  // s - P (mod 2^64)
    return (s < a || s >= P) ? t : s;
}
FR_HD uint64_t gl_sub(uint64_t a, uint64_t b) {
    uint64_t d = a - b;
    return a < b ? d - EPS : d;  // + P
}
FR_HD uint64_t gl_neg(uint64_t a) { return a ? P - a : 0; }

// 64x64 -> 128 from four 32x32->64 products (v_mad_u64_u32 on gfx950)
FR_HD void mul64wide(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
    uint64_t a0 = (uint32_t)a, a1 = a >> 32, b0 = (uint32_t)b, b1 = b >> 32;
    uint64_t p00 = a0 * b0;
    uint64_t mid = a0 * b1 + (p00 >> 32);            // < 2^64
    uint64_t mid2 = a1 * b0 + (uint32_t)mid;         // < 2^64
    lo = (mid2 << 32) | (uint32_t)p00;
    hi = a1 * b1 + (mid >> 32) + (mid2 >> 32);
}
// reduce hi*2^64 + lo mod P (canonical)
FR_HD uint64_t gl_reduce(uint64_t hi, uint64_t lo) {
    uint64_t hh = hi >> 32, hl = (uint32_t)hi;
    uint64_t t = lo - hh;
    if (lo < hh) t -= EPS;
    uint64_t u = (hl << 32) - hl;  // hl * (2^32 - 1)
    uint64_t r = t + u;
    if (r < t) r += EPS;
    return r >= P ? r - P : r;
}
FR_HD uint64_t gl_mul(uint64_t a, uint64_t b) {
    uint64_t hi, lo;
    mul64wide(a, b, hi, lo);
    return gl_reduce(hi, lo);
}
inline uint64_t gl_pow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = gl_mul(r, b);
        b = gl_mul(b, b);
        e >>= 1;
    }
    return r;
}

// PBS gadget decomposition of a canonical x: round(x / g) in [0, 2^23],
// recentred to [-2^22, 2^22) and returned as an element of Z_p.
FR_HD uint64_t pbs_decompose(uint64_t x) {
    uint64_t w = (x >> 9) + 0x7FFFFFFFULL + (((x & 511) + 256) >> 9);  // floor((x + g/2) / 2^9)
    uint64_t q = w >> 32;
    uint64_t rem = (uint32_t)w + q;
    if (rem >= EPS) q += 1;                                            // floor(w / (2^32 - 1))
    return q >= (1ULL << 22) ? P - ((1ULL << 23) - q) : q;
}

// Z_p -> torus 2^64: round(x * 2^64 / P) for canonical x.
FR_HD uint64_t zp_to_torus(uint64_t x) {
    // x*2^64 = x*P + x*(2^32-1); v = x*(2^32-1) + (P-1)/2 (128-bit)
    uint64_t vhi = x >> 32, vlo = x << 32;
    uint64_t nlo = vlo - x;
    vhi -= (vlo < x) ? 1 : 0;
    const uint64_t half = (P - 1) / 2;
    uint64_t lo2 = nlo + half;
    vhi += (lo2 < nlo) ? 1 : 0;
    // q = floor(v / P), start from vhi; r = v - vhi*P = lo2 + vhi*(2^32-1)  (< 2^65)
    uint64_t q = vhi;
    uint64_t add = (vhi << 32) - vhi;
    uint64_t r = lo2 + add;
    uint64_t rc = (r < lo2) ? 1 : 0;  // carry bit (value rc*2^64 + r)
    // subtract P while >= P
    for (int it = 0; it < 3; ++it) {
        bool ge = rc || r >= P;
        if (!ge) break;
        uint64_t nr = r - P;
        rc = rc - ((r < P) ? 1 : 0);
        r = nr;
        q += 1;
    }
    return x + q;
}

}  // namespace fr
