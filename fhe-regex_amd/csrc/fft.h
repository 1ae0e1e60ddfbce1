// The torus ring of the blind rotation: T_64[X]/(X^N+1) (coefficients mod
// 2^64, as in tfhe-rs), polynomial products through an f64 negacyclic FFT —
// the same representation tfhe-rs 0.2 uses for its Fourier bootstrapping key
// (reference Cargo.lock:602-615, concrete-fft 0.1.0 at Cargo.lock:110-114).
//
// Transform: a real polynomial a of degree < N folds into M = N/2 complex
// points z_k = a_k + i a_(k+M), i.e. a mod (x^M - i) with x^M = i.  The M roots
// of x^M - i are psi^L (psi = e^(i pi / N), L = 1 mod 4); the forward
// transform is the merged-twiddle Cooley-Tukey split of x^M - i:
//   node (s, b) holds z mod (x^(M/2^s) - psi^E(s,b)),  E(0,0) = M,
//   children E/2 and E/2 + N (mod 2N), butterfly twiddle c = psi^(E/2):
//       (lo, hi) -> (lo + c hi, lo - c hi)                       (forward)
//       (A, B)   -> (A + B, conj(c) (A - B))   (inverse, times 2 per stage)
// so after log2 M stages slot j holds a(psi^L(j)) with L(j) = E(log2 M, j).
// The inverse therefore returns M * z; the 1/M = 2^-log2(M) factor (exact in
// f64) is folded into the Fourier bootstrapping key.  Multiplying by X^e is
// the slot-wise factor psi^(e L(j) mod 2N).
//
// Every floating-point step is a fixed sequence of IEEE-754 double operations
// (mul, add, fma; -ffp-contract=off everywhere), so the device kernel, the
// host key transform and oracle/tfhe_oracle.c's restatement agree bit for bit.
// Twiddles are computed once on the host (psi_pow) and uploaded.
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>

#include "common.h"

namespace fr {
namespace fft {

struct c64 {
    double re, im;
};

#if defined(__HIPCC__)
#define FR_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#define FR_FMA(a, b, c) std::fma((a), (b), (c))
#endif

// a * b: re = fma(a.re, b.re, -(a.im b.im)), im = fma(a.re, b.im, a.im b.re)
FR_HD void cmul(double ar, double ai, double br, double bi, double& zr, double& zi) {
    const double pr = -(ai * bi), pi = ai * br;
    zr = FR_FMA(ar, br, pr);
    zi = FR_FMA(ar, bi, pi);
}
// z += a * b: re = fma(-a.im, b.im, fma(a.re, b.re, z.re)), im = fma(a.im, b.re, fma(a.re, b.im, z.im))
FR_HD void cmac(double ar, double ai, double br, double bi, double& zr, double& zi) {
    zr = FR_FMA(-ai, bi, FR_FMA(ar, br, zr));
    zi = FR_FMA(ai, br, FR_FMA(ar, bi, zi));
}
// forward butterfly (lo, hi) <- (lo + c hi, lo - c hi) in six fused operations:
//   lo' = (fma(c.re, hi.re, fma(-c.im, hi.im, lo.re)), fma(c.re, hi.im, fma(c.im, hi.re, lo.im)))
//   hi' = 2 lo - lo' = (fma(2, lo.re, -lo'.re), fma(2, lo.im, -lo'.im))
// (the absolute error of hi' is that of lo', one rounding of |lo| + |c hi|)
FR_HD void fwd_bf(double& xr, double& xi, double& yr, double& yi, double cr, double ci) {
    const double ur = FR_FMA(cr, yr, FR_FMA(-ci, yi, xr));
    const double ui = FR_FMA(cr, yi, FR_FMA(ci, yr, xi));
    yr = FR_FMA(2.0, xr, -ur);
    yi = FR_FMA(2.0, xi, -ui);
    xr = ur;
    xi = ui;
}
// inverse butterfly: d = u - v; (u, v) <- (u + v, conj(c) * d)
//   conj(c) d: re = fma(c.re, d.re, c.im d.im), im = fma(c.re, d.im, -(c.im d.re))
FR_HD void inv_bf(double& ur, double& ui, double& vr, double& vi, double cr, double ci) {
    const double dr = ur - vr, di = ui - vi;
    ur = ur + vr;
    ui = ui + vi;
    const double pr = ci * di, pi = -(ci * dr);
    vr = FR_FMA(cr, dr, pr);
    vi = FR_FMA(cr, di, pi);
}
// inverse radix-4 group: stages s1 = 2p + 1 then s0 = 2p of an even-log2(M) inverse
// transform on x0..x3 (x1 = x0's stage-s1 partner, x2 = its stage-s0 partner).  Stage
// s1's twiddles are ca and i ca (siblings of the split tree, fft::Tables), stage s0's c:
//   a = x0 + x1, d1 = x0 - x1, b = x2 + x3, d2 = x2 - x3,
//   t1 = d1 - i d2, t2 = d1 + i d2                      (exact swaps and signs)
//   x0 <- a + b, x1 <- conj(ca) t1, x2 <- conj(c) (a - b), x3 <- conj(cc) t2
// with cc = c ca (cmul) and conj(w) d as in inv_bf: 28 operations for 4 x inv_bf's 32
FR_HD void inv_r4(double& x0r, double& x0i, double& x1r, double& x1i, double& x2r, double& x2i, double& x3r,
                  double& x3i, double cr, double ci, double car, double cai, double ccr, double cci) {
    const double ar = x0r + x1r, ai = x0i + x1i, d1r = x0r - x1r, d1i = x0i - x1i;
    const double br = x2r + x3r, bi = x2i + x3i, d2r = x2r - x3r, d2i = x2i - x3i;
    const double t1r = d1r + d2i, t1i = d1i - d2r, t2r = d1r - d2i, t2i = d1i + d2r;
    const double er = ar - br, ei = ai - bi;
    x0r = ar + br;
    x0i = ai + bi;
    x1r = FR_FMA(car, t1r, cai * t1i);
    x1i = FR_FMA(car, t1i, -(cai * t1r));
    x2r = FR_FMA(cr, er, ci * ei);
    x2i = FR_FMA(cr, ei, -(ci * er));
    x3r = FR_FMA(ccr, t2r, cci * t2i);
    x3i = FR_FMA(ccr, t2i, -(cci * t2r));
}
// psi^k (k in [0, 2N)) from the quadrant table qt[r] = psi^r, r < N/2:
// psi^k = i^(k / (N/2)) psi^(k mod N/2); i * (a + bi) = -b + ai.
FR_HD void psi_quadrant(double ar, double ai, uint32_t q, double& zr, double& zi) {
    if (q & 1) {
        const double t = ar;
        ar = -ai;
        ai = t;
    }
    if (q & 2) {
        ar = -ar;
        ai = -ai;
    }
    zr = ar;
    zi = ai;
}
// f64 (an integer-valued approximation, |v| < 2^100) -> rint(v) mod 2^64 (round
// half to even), exact: ri = rint(v); hi = floor(ri / 2^32); lo = ri - hi 2^32 in
// [0, 2^32); hi mod 2^32 = hi - floor(hi / 2^32) 2^32.  Every step is exact, so
// this equals any other exact evaluation of rint(v) mod 2^64 (oracle/tfhe_oracle.c
// reduces by 2^64 first).
FR_HD uint64_t torus_of(double v) {
#if defined(__HIPCC__)
    const double ri = __builtin_rint(v);
    const double hi = __builtin_floor(ri * 0x1p-32);
    const double hm = FR_FMA(-__builtin_floor(hi * 0x1p-32), 0x1p32, hi);
#else
    const double ri = std::nearbyint(v);
    const double hi = std::floor(ri * 0x1p-32);
    const double hm = FR_FMA(-std::floor(hi * 0x1p-32), 0x1p32, hi);
#endif
    const double lo = FR_FMA(-hi, 0x1p32, ri);
    return ((uint64_t)(uint32_t)hm << 32) | (uint64_t)(uint32_t)lo;
}
// The blind rotation's accumulator is f64: a torus value a (mod 2^64) is held as
// t = a 2^-ACC_LOG, a double in [-2^22, 2^22] (ACC_LOG = 41 = 64 - B for the one-level
// gadget base 2^B = 2^23) congruent to a 2^-ACC_LOG up to the rounding of the additions
// (below 2^44 2^-ACC_LOG per step, far under the bootstrap noise).  The
// Fourier key carries the same 2^-ACC_LOG (with the transform's 1/M), so every product
// and sum of a step is the unscaled computation times an exact power of two: the same
// mantissas, the same roundings (no value comes near the f64 range limits).  Per step:
//   digit  d = rint(t) in [-2^(B-1), 2^(B-1)] (the closest multiple of 2^(64-B) of a,
//          ties to even)
//   update t = reduce(t + v), v the inverse transform's f64 output (|v| < 2^59),
//          reduce(t) = fma(-rint(t 2^-B), 2^B, t), exact
// and torus_of(t 2^ACC_LOG) gives the u64 torus value for sample extraction.
// (Round 3 held a itself: digit rint(a 2^-41), reduce by 2^64; the scaled form saves the
// digit's multiply, 8 VALU per lane and step of the latency shape.)
#if defined(__HIPCC__)
#define FR_RINT(x) __builtin_rint(x)
#else
#define FR_RINT(x) std::nearbyint(x)
#endif
constexpr int ACC_LOG = 41;
template <int B>
FR_HD double acc_digit(double t) {
    static_assert(B == 64 - ACC_LOG, "the accumulator unit is the gadget's 2^(64-B)");
    return FR_RINT(t);
}
template <int B>
FR_HD double acc_reduce(double t) {
    static_assert(B == 64 - ACC_LOG, "the accumulator unit is the gadget's 2^(64-B)");
    return FR_FMA(-FR_RINT(t * (1.0 / (double)(1ULL << B))), (double)(1ULL << B), t);
}
// exact f64 of a u64 torus value (signed representative in [-2^63, 2^63)), in accumulator units
FR_HD double acc_of_torus(uint64_t u) { return (double)(int64_t)u * 0x1p-41; }
// the u64 torus value of an accumulator entry
FR_HD uint64_t torus_of_acc(double t) { return torus_of(t * 0x1p41); }
// scale of the Fourier bootstrapping key: the inverse transform's 1/M and the accumulator unit
FR_HD double fourier_key_scale(int log2M) {
#if defined(__HIPCC__)
    return __builtin_ldexp(1.0, -(log2M + ACC_LOG));
#else
    return std::ldexp(1.0, -(log2M + ACC_LOG));
#endif
}

// ---------------------------------------------------------------- host side
// psi^x (x mod 2N) = i^q (cos(pi r / N), sin(pi r / N)), x = q N/2 + r
c64 psi_pow(int N, int64_t x);

struct Tables {
    int N = 0, M = 0, LOG = 0;
    std::vector<c64> tw;      // [M]: tw[(1 << s) + b] = psi^(E(s,b)/2); tw[0] unused
    std::vector<c64> qt;      // [N/2]: psi^r
    std::vector<uint16_t> leaf;  // [M]: L(j) = E(LOG, j) mod 2N
    explicit Tables(int N);
    void forward(c64* z) const;   // natural order -> slot order (M points)
    void inverse(c64* z) const;   // slot order -> natural order, times M (radix-4 pairs, LOG even)
};

// Fourier bootstrapping key: every GGSW polynomial of the torus BSK
// ([w][r][c][coef] u64) folded, transformed and scaled by fourier_key_scale (1/M and the
// accumulator unit 2^-ACC_LOG), as [w][r][c][slot] complex.
void bsk_to_fourier(const Tables& T, const std::vector<uint64_t>& bsk, size_t polys, std::vector<c64>& out);

}  // namespace fft
}  // namespace fr
