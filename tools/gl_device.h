// Device-side Goldilocks arithmetic with non-canonical intermediates.
//
// Values live in [0, 2^64) and are only reduced to [0, P) where a canonical
// representative is required (gadget decomposition, output).  Carries come
// from the add/sub-with-carry builtins so the compiler emits v_add_co /
// v_addc_co / v_sub_co / v_subb_co chains instead of 64-bit compares.
#pragma once
#include <cstdint>

#include "goldilocks.h"

namespace fr {
namespace gd {

typedef unsigned long long u64c;

// 128-bit product from four v_mad_u64_u32
__device__ __forceinline__ void mulw(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
    const uint64_t a0 = (uint32_t)a, a1 = a >> 32, b0 = (uint32_t)b, b1 = b >> 32;
    const uint64_t p00 = a0 * b0;
    const uint64_t t1 = a0 * b1 + (p00 >> 32);
    const uint64_t t2 = a1 * b0 + (uint32_t)t1;
    hi = a1 * b1 + ((t1 >> 32) + (t2 >> 32));
    lo = (t2 << 32) | (uint32_t)p00;
}
// hi*2^64 + lo (mod P) -> [0, 2^64):  lo - h1 + h0*(2^32-1), with the two
// wrap-arounds corrected by -/+ (2^32-1).
__device__ __forceinline__ uint64_t red(uint64_t hi, uint64_t lo) {
    const uint32_t h0 = (uint32_t)hi, h1 = (uint32_t)(hi >> 32);
    u64c c1, c2;
    const uint64_t s = __builtin_subcll(lo, (uint64_t)h1, 0ULL, &c1);
    const uint64_t u = ((uint64_t)h0 << 32) - h0;
    uint64_t r = __builtin_addcll(s, u, 0ULL, &c2);
    r += c2 ? EPS : 0;
    r -= c1 ? EPS : 0;
    return r;
}
__device__ __forceinline__ uint64_t mul(uint64_t a, uint64_t b) {
    uint64_t hi, lo;
    mulw(a, b, hi, lo);
    return red(hi, lo);
}
// [0, 2^64) -> [0, P): t + (2^32-1) carries out iff t >= P
__device__ __forceinline__ uint64_t canon(uint64_t t) {
    u64c c;
    const uint64_t t2 = __builtin_addcll(t, EPS, 0ULL, &c);
    return c ? t2 : t;
}
// x + t and x - t for any x and canonical t (no second wrap possible)
__device__ __forceinline__ uint64_t add_c(uint64_t x, uint64_t t) {
    u64c c;
    const uint64_t s = __builtin_addcll(x, t, 0ULL, &c);
    return s + (c ? EPS : 0);
}
__device__ __forceinline__ uint64_t sub_c(uint64_t x, uint64_t t) {
    u64c b;
    const uint64_t d = __builtin_subcll(x, t, 0ULL, &b);
    return d - (b ? EPS : 0);
}
// x + y and x - y for any x, y (a second wrap is possible and corrected)
__device__ __forceinline__ uint64_t add_g(uint64_t x, uint64_t y) {
    u64c c, c2;
    const uint64_t s = __builtin_addcll(x, y, 0ULL, &c);
    const uint64_t s2 = __builtin_addcll(s, c ? EPS : 0, 0ULL, &c2);
    return s2 + (c2 ? EPS : 0);
}
__device__ __forceinline__ uint64_t sub_g(uint64_t x, uint64_t y) {
    u64c b, b2;
    const uint64_t d = __builtin_subcll(x, y, 0ULL, &b);
    const uint64_t d2 = __builtin_subcll(d, b ? EPS : 0, 0ULL, &b2);
    return d2 - (b2 ? EPS : 0);
}
// forward (Cooley-Tukey) butterfly: (x, y) -> (x + z*y, x - z*y)
__device__ __forceinline__ void ct(uint64_t& x, uint64_t& y, uint64_t z) {
    const uint64_t t = canon(mul(z, y));
    y = sub_c(x, t);
    x = add_c(x, t);
}
// inverse (Gentleman-Sande) butterfly with the flipped twiddle:
// (u, v) -> (u + v, (v - u) * z'),  z' = -zeta^-1 (see NttGeo)
__device__ __forceinline__ void gs(uint64_t& u, uint64_t& v, uint64_t z) {
    const uint64_t d = sub_g(v, u);
    u = add_g(u, v);
    v = mul(d, z);
}


// ---- variant 2: explicit 32-bit carry chains --------------------------------
__device__ __forceinline__ void mulw2(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0, p01 = (uint64_t)a0 * b1, p10 = (uint64_t)a1 * b0, p11 = (uint64_t)a1 * b1;
    unsigned c1, c2, c3, c4;
    uint32_t m = __builtin_addc((uint32_t)(p00 >> 32), (uint32_t)p01, 0u, &c1);
    m = __builtin_addc(m, (uint32_t)p10, 0u, &c2);
    uint32_t h0 = __builtin_addc((uint32_t)p11, (uint32_t)(p01 >> 32), c1, &c3);
    h0 = __builtin_addc(h0, (uint32_t)(p10 >> 32), c2, &c4);
    const uint32_t h1 = (uint32_t)(p11 >> 32) + c3 + c4;
    lo = ((uint64_t)m << 32) | (uint32_t)p00;
    hi = ((uint64_t)h1 << 32) | h0;
}
// hi*2^64 + lo = lo + hl*2^32 - (hh + hl)  (mod P); one net +-(2^32-1) fix-up
__device__ __forceinline__ uint64_t red2(uint64_t hi, uint64_t lo) {
    const uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32), hl = (uint32_t)hi, hh = (uint32_t)(hi >> 32);
    unsigned c1, cs, b1, b2;
    const uint32_t u1 = __builtin_addc(l1, hl, 0u, &c1);  // u = lo + hl*2^32 (carry c1 = 2^64)
    const uint32_t s0 = __builtin_addc(hh, hl, 0u, &cs);  // S = hh + hl (33 bits)
    const uint32_t r0 = __builtin_subc(l0, s0, 0u, &b1);
    const uint32_t r1 = __builtin_subc(u1, cs, b1, &b2);  // r = u - S (borrow b2 = -2^64)
    const uint64_t r = ((uint64_t)r1 << 32) | r0;
    const uint64_t d = (c1 & ~b2) ? EPS : ((b2 & ~c1) ? (0ULL - EPS) : 0ULL);
    return r + d;
}
__device__ __forceinline__ uint64_t mul2(uint64_t a, uint64_t b) {
    uint64_t hi, lo;
    mulw2(a, b, hi, lo);
    return red2(hi, lo);
}
// x + t, t canonical: single wrap corrected by + (2^32-1)
__device__ __forceinline__ uint64_t add_c2(uint64_t x, uint64_t t) {
    unsigned c0, c;
    const uint32_t s0 = __builtin_addc((uint32_t)x, (uint32_t)t, 0u, &c0);
    const uint32_t s1 = __builtin_addc((uint32_t)(x >> 32), (uint32_t)(t >> 32), c0, &c);
    return (((uint64_t)s1 << 32) | s0) + (c ? EPS : 0ULL);
}
__device__ __forceinline__ uint64_t sub_c2(uint64_t x, uint64_t t) {
    unsigned b0, b;
    const uint32_t d0 = __builtin_subc((uint32_t)x, (uint32_t)t, 0u, &b0);
    const uint32_t d1 = __builtin_subc((uint32_t)(x >> 32), (uint32_t)(t >> 32), b0, &b);
    return (((uint64_t)d1 << 32) | d0) - (b ? EPS : 0ULL);
}
__device__ __forceinline__ void ct2(uint64_t& x, uint64_t& y, uint64_t z) {
    const uint64_t t = canon(mul2(z, y));
    y = sub_c2(x, t);
    x = add_c2(x, t);
}
__device__ __forceinline__ void gs2(uint64_t& u, uint64_t& v, uint64_t z) {
    const uint64_t d = sub_g(v, u);
    u = add_g(u, v);
    v = mul2(d, z);
}

}  // namespace gd
}  // namespace fr
