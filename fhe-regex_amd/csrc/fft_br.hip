// Blind rotation on the 2^64 torus with an f64 negacyclic FFT (FR_RING_FFT),
// gfx950.  The ring, the transform and every floating-point operation are
// specified in fft.h; oracle/tfhe_oracle.c restates the same sequence.
// (File named fft_br.hip so its object does not collide with fft.cpp.)
//
//   k_blind_rotate_fft<N,E>: modulus switch, test-polynomial accumulator (u64),
//     the unrolled blind rotation (k = 1: one step per pair of LWE
//     coefficients, three GGSWs, see device.hip), multi-value w-step and
//     sample extract -- outputs are already torus LWEs, no ring conversion.
//
// Geometry: one workgroup per bootstrap, 2 * M/E lanes (M = N/2 complex
// points per polynomial, E per lane, whole waves per polynomial).  The
// log2 M transform stages run as register phases of log2 E stages joined by
// LDS exchanges of 16-B complex values (conflict-free maps of geo.h with
// 8-lane b128 groups).  Per step a lane: gadget digits of its 2E accumulator
// coefficients (local, exact), forward FFT, MAC with the three Fourier GGSWs
// (coalesced [w][r][c][m][lane] layout) and their slot-wise monomial factors
// psi^(e L) - 1 (quadrant table in LDS), inverse FFT, exact f64 -> torus
// conversion and u64 accumulate.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstring>

#include "device.h"
#include "fft.h"
#include "geo.h"

namespace fr {

#define FFT_CHECK(x)                                                                         \
    do {                                                                                     \
        hipError_t _e = (x);                                                                 \
        if (_e != hipSuccess)                                                                \
            throw Error(FR_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(_e) +     \
                                        " at " __FILE__ ":" + std::to_string(__LINE__));     \
    } while (0)

template <int M, int E>
using FGeo = NttGeo<M, E, 3, fft_layout_variant(ilog2c(M), ilog2c(E))>;
template <int M, int E>
constexpr int FV = fft_layout_variant(ilog2c(M), ilog2c(E));

// FR_BR_TIMING (debug builds only): wave 0 of workgroup 0 accumulates
// s_memtime deltas of the step segments and prints them at the end.
#ifdef FR_BR_TIMING
#define FBR_STAMP(k)                                            \
    do {                                                        \
        __builtin_amdgcn_sched_barrier(0);                      \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
        tseg[k] += now_ - tlast;                                \
        tlast = now_;                                           \
        __builtin_amdgcn_sched_barrier(0);                      \
    } while (0)
#else
#define FBR_STAMP(k) \
    do {             \
    } while (0)
#endif

__device__ __forceinline__ void cfwd(double2& x, double2& y, double2 c) { fft::fwd_bf(x.x, x.y, y.x, y.y, c.x, c.y); }
__device__ __forceinline__ void cinv(double2& u, double2& v, double2 c) { fft::inv_bf(u.x, u.y, v.x, v.y, c.x, c.y); }

// k = 1 (log2 M even, E = 4): every phase is two stages s0 = 2p, s1 = 2p + 1 and the
// inverse takes them as one radix-4 group (fft.h inv_r4).  A lane's twiddles of such a
// phase are c (stage s0, both pairs), ca (stage s1, pair 0/1; pair 2/3 has i ca exactly,
// fft::Tables) and cc = c ca (inverse only).
template <int M, int E>
constexpr bool fradix4() {
    return E == 4 && FGeo<M, E>::LOG % 2 == 0;
}
template <int M, int E>
struct FTwr {
    static constexpr int COUNT = fradix4<M, E>() ? FGeo<M, E>::NPH * 3 : FGeo<M, E>::LOG * (E / 2);
    double2 v[COUNT];
};
// i c (exact: a swap and a sign)
__device__ __forceinline__ double2 fmul_i(double2 c) { return make_double2(-c.y, c.x); }
__device__ __forceinline__ void cinv_r4(double2 (&x)[4], double2 c, double2 ca, double2 cc) {
    fft::inv_r4(x[0].x, x[0].y, x[1].x, x[1].y, x[2].x, x[2].y, x[3].x, x[3].y, c.x, c.y, ca.x, ca.y, cc.x, cc.y);
}
// the radix-4 twiddles (c, ca) of phase p for this lane from the LDS table
template <int M, int E, int p>
__device__ __forceinline__ void ftw_r4(const double2* tw, int tl, double2& c, double2& ca) {
    using G = FGeo<M, E>;
    constexpr int s0 = G::s_begin(p), s1 = s0 + 1;
    const int b = G::template base<p>(tl);
    c = (tw + (b >> (G::LOG - s0)))[(1 << s0) + (G::template moff<p>(0) >> (G::LOG - s0))];
    ca = (tw + (b >> (G::LOG - s1)))[(1 << s1) + (G::template moff<p>(0) >> (G::LOG - s1))];
}

template <int M, int E, int p>
__device__ __forceinline__ void ffwd_phase(double2 (&x)[E], const double2* tw, int tl) {
    using G = FGeo<M, E>;
    const int b = G::template base<p>(tl);
#pragma unroll
    for (int s = G::s_begin(p); s < G::s_end(p); ++s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
        const double2* zs = tw + (b >> (G::LOG - s));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            cfwd(x[m], x[m + dm], zs[(1 << s) + (G::template moff<p>(m) >> (G::LOG - s))]);
        }
    }
}
template <int M, int E, int p>
__device__ __forceinline__ void finv_phase(double2 (&x)[E], const double2* tw, int tl);
// (radix-4 phases: cc = c ca from the product table twc, indexed like c)
template <int M, int E, int p>
__device__ __forceinline__ void finv_phase_lds(double2 (&x)[E], const double2* tw, const double2* twc, int tl) {
    if constexpr (fradix4<M, E>()) {
        using G = FGeo<M, E>;
        constexpr int s0 = G::s_begin(p);
        double2 c, ca;
        ftw_r4<M, E, p>(tw, tl, c, ca);
        const double2 cc = (twc + (G::template base<p>(tl) >> (G::LOG - s0)))[(1 << s0) + (G::template moff<p>(0) >> (G::LOG - s0))];
        cinv_r4(x, c, ca, cc);
    } else {
        finv_phase<M, E, p>(x, tw, tl);
    }
}
template <int M, int E, int p>
__device__ __forceinline__ void finv_phase(double2 (&x)[E], const double2* tw, int tl) {
    using G = FGeo<M, E>;
    const int b = G::template base<p>(tl);
#pragma unroll
    for (int s = G::s_end(p) - 1; s >= G::s_begin(p); --s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
        const double2* zs = tw + (b >> (G::LOG - s));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            cinv(x[m], x[m + dm], zs[(1 << s) + (G::template moff<p>(m) >> (G::LOG - s))]);
        }
    }
}

// Latency shape: a lane's twiddles are the same every step (they depend on the
// lane, the stage and the element only), so they are read from LDS once and
// kept in registers: LOG * E / 2 complex values, index (s, k-th butterfly of s).
// phases of the latency shape's forward FFT after which its 2nd and 3rd non-prefetched GGSW groups load
#ifndef FR_LAT_LOAD1
#define FR_LAT_LOAD1 2
#endif
#ifndef FR_LAT_LOAD2
#define FR_LAT_LOAD2 3
#endif
// latency shape: how many of a step's three GGSW groups are loaded right after the
// previous step's MAC (the rest across the step's own forward FFT)
#ifndef FR_LAT_PF
#define FR_LAT_PF 2
#endif
// the same for k = 2 (tools/ab_k2.sh: 0 / 1 / 2 / 3 groups: one bootstrap 1.75 / 1.71 / 1.67 / 1.81 ms)
#ifndef FR_LAT_PF2
#define FR_LAT_PF2 2
#endif
// pair shape: the forward phase after which a step's third GGSW group loads (tools/ab_libs.sh,
// profiles/r03/ab_pair_variants.log: after phase 0 / 1 / 2 / 3: 2.93 / 2.83 / 2.73 / 2.82 ms per
// 512 bootstraps; the psi lookups moved ahead of the MAC barrier: 2.75, not kept)
#ifndef FR_PAIR_LOAD
#define FR_PAIR_LOAD 2
#endif
// pair shape A/B knobs: key groups loaded a step ahead (FR_PAIR_PF; with 1 the third group
// loads after forward phase FR_PAIR_LOAD2), and the inverse's c ca recomputed per phase (1) or
// kept (0).  Round 4 (profiles/r04/ab_key_placement{,2,3}.log, 512 / 2048 bootstraps): one group
// ahead, the second after forward phase 2 and the third after phase 4 (in the MAC barrier's
// shadow, its registers free across the transform) 2.66-2.67 / 9.48-9.51 ms, against 2.72-2.75 /
// 9.81-9.83 for two groups ahead and the third after phase 2; the third after phase 3: 9.65-9.67
#ifndef FR_PAIR_PF
#define FR_PAIR_PF 1
#endif
#ifndef FR_PAIR_LOAD2
#define FR_PAIR_LOAD2 4
#endif
#ifndef FR_PAIR_CC
#define FR_PAIR_CC 1
#endif
// latency shape: the MAC's key-only part and own-row product before the MAC barrier, the next
// step's key prefetch with them (1), or all of the MAC after the barrier (0)
#ifndef FR_MAC_EARLY
#define FR_MAC_EARLY 0
#endif
// latency shape, k = 1: the lane's twiddles in registers (1) or read from LDS (0)
#ifndef FR_LAT_TWR
#define FR_LAT_TWR 1
#endif
// Round-3 latency-shape experiments, measured and not kept (logs under profiles/r03/):
//  * per-polynomial synchronisation: LDS arrival counters in place of the workgroup
//    barriers around each polynomial's cross-wave exchanges, and the MAC waiting for the
//    other polynomial only where it reads it: 1.49 against 1.34 ms per bootstrap, at any
//    start skew; the late MAC wait alone: 1.35 (ab_poly_sync.log);
//  * the MAC's key products computed in the shadow of the forward cross-wave exchange,
//    the next step's key loaded right after them: 1.38 ms (ab_kearly.log);
//  * k = 1 throughput shapes with E = 8 / 16 (two waves / one wave per polynomial): 12.0 /
//    13.4 against 10.8 ms per 2048 bootstraps (ab_lane_elems_k1.log);
//  * a 16-wave latency shape (E = 2, build with -DFR_LAT_E2): 2.03 ms with the twiddles
//    from LDS, 2.27 with them in registers (spilled at the 128-VGPR cap of 4 waves per
//    SIMD), against 1.34: nine exchanges per transform, three of them cross-wave
//    (ab_lat_e2_16wave.log).

// The twiddles of phase p are wave-uniform when every lane of a wave reads the same table
// entry for each of the phase's stages (the index bits the entry depends on sit on element or
// wave bits of that layout: phases 0 and 1 of the k = 1 geometry).  Those stay in SGPRs, which
// frees 4 VGPRs per complex twiddle (pair shape: 16 of its 256, where it spilled 16).
template <int M, int E, int p>
constexpr bool ftw_wave_uniform() {
    using G = FGeo<M, E>;
    for (int w = 0; w * 64 < G::T; ++w)
        for (int s = G::s_begin(p); s < G::s_end(p); ++s) {
            const int ref = geo_base(G::LOG, G::e, p, w * 64, FV<M, E>) >> (G::LOG - s);
            for (int l = 1; l < 64; ++l)
                if ((geo_base(G::LOG, G::e, p, w * 64 + l, FV<M, E>) >> (G::LOG - s)) != ref) return false;
        }
    return true;
}
__device__ __forceinline__ double2 fwave_uniform(double2 v) {
    const unsigned long long a = (unsigned long long)__double_as_longlong(v.x);
    const unsigned long long b = (unsigned long long)__double_as_longlong(v.y);
    const unsigned a0 = __builtin_amdgcn_readfirstlane((unsigned)a), a1 = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const unsigned b0 = __builtin_amdgcn_readfirstlane((unsigned)b), b1 = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return make_double2(__longlong_as_double((long long)(((unsigned long long)a1 << 32) | a0)),
                        __longlong_as_double((long long)(((unsigned long long)b1 << 32) | b0)));
}
// Measured (profiles/r04/ab_r04c.log): the pair shape gains (512 bootstraps 2.62-2.69 -> 2.53-2.56 ms,
// its 16 spilled VGPRs gone); the latency shape lost 5% (one bootstrap 1.31 -> 1.38 ms, a worse
// schedule at 190 VGPRs), so it keeps the twiddles in VGPRs
#ifndef FR_TW_SGPR_PAIR
#define FR_TW_SGPR_PAIR 1
#endif
#ifndef FR_TW_SGPR_LAT
#define FR_TW_SGPR_LAT 0
#endif

template <int M, int E>
constexpr int ftw_index(int s, int m) {
    const int d = FGeo<M, E>::LOG - 1 - s - FGeo<M, E>::lo(s / FGeo<M, E>::e);
    return s * (E / 2) + ((m >> (d + 1)) << d) + (m & ((1 << d) - 1));
}
template <int M, int E, int p, bool UNI = false>
__device__ __forceinline__ void ftw_load_phase(FTwr<M, E>& twr, const double2* tw, int tl) {
    using G = FGeo<M, E>;
    if constexpr (fradix4<M, E>()) {
        double2 c, ca, cc;
        ftw_r4<M, E, p>(tw, tl, c, ca);
        fft::cmul(c.x, c.y, ca.x, ca.y, cc.x, cc.y);
        if constexpr (UNI && ftw_wave_uniform<M, E, p>()) {
            c = fwave_uniform(c);
            ca = fwave_uniform(ca);
            cc = fwave_uniform(cc);
        }
        twr.v[3 * p] = c, twr.v[3 * p + 1] = ca, twr.v[3 * p + 2] = cc;
        if constexpr (p + 1 < G::NPH) ftw_load_phase<M, E, p + 1, UNI>(twr, tw, tl);
        return;
    }
    const int b = G::template base<p>(tl);
#pragma unroll
    for (int s = G::s_begin(p); s < G::s_end(p); ++s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
        const double2* zs = tw + (b >> (G::LOG - s));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            twr.v[ftw_index<M, E>(s, m)] = zs[(1 << s) + (G::template moff<p>(m) >> (G::LOG - s))];
        }
    }
    if constexpr (p + 1 < G::NPH) ftw_load_phase<M, E, p + 1, UNI>(twr, tw, tl);
}
template <int M, int E, int p>
__device__ __forceinline__ void ffwd_phase_r(double2 (&x)[E], const FTwr<M, E>& twr) {
    using G = FGeo<M, E>;
    if constexpr (fradix4<M, E>()) {  // stage s0: pairs (0, 2), (1, 3); stage s1: (0, 1), (2, 3)
        const double2 c = twr.v[3 * p], ca = twr.v[3 * p + 1];
        cfwd(x[0], x[2], c);
        cfwd(x[1], x[3], c);
        cfwd(x[0], x[1], ca);
        cfwd(x[2], x[3], fmul_i(ca));
        return;
    }
#pragma unroll
    for (int s = G::s_begin(p); s < G::s_end(p); ++s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            cfwd(x[m], x[m + dm], twr.v[ftw_index<M, E>(s, m)]);
        }
    }
}
template <int M, int E, int p>
__device__ __forceinline__ void finv_phase_r(double2 (&x)[E], const FTwr<M, E>& twr) {
    using G = FGeo<M, E>;
    if constexpr (fradix4<M, E>()) {
        cinv_r4(x, twr.v[3 * p], twr.v[3 * p + 1], twr.v[3 * p + 2]);
        return;
    }
#pragma unroll
    for (int s = G::s_end(p) - 1; s >= G::s_begin(p); --s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            cinv(x[m], x[m + dm], twr.v[ftw_index<M, E>(s, m)]);
        }
    }
}

// exchange between phase layouts stays inside each wave (see device.hip)
template <int M, int E, int PF, int PT>
constexpr bool fwave_local() {
    using G = FGeo<M, E>;
    for (int b = 6; (1 << b) < G::T; ++b)
        if (G::lane_bit(PF, b) != G::lane_bit(PT, b)) return false;
    return true;
}
__device__ __forceinline__ void fwave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Register exchanges.  An exchange between adjacent layouts transposes the lane's
// element bits with the lane bits that carry the arriving index bits.  When element
// bit j leaves through the same lane bit k that brings in the next layout's element
// bit j, and k is 4 or 5 (row pairs / wave halves), the transpose of each pair
// (A = x[m], B = x[m | 2^j]) is one v_permlane16/32_swap per dword: lanes with bit k
// clear keep A and receive the partner's A as B; lanes with bit k set keep B and
// receive the partner's B as A.  No LDS traffic and no barrier (E = 4: the exchange
// between layouts 1 and 2 of both transforms).
template <int M, int E, int PF, int PT>
constexpr int fperm_lane_bit(int j) {
    using G = FGeo<M, E>;
    const int out = G::lo(PF) + j, in = G::lo(PT) + j;
    int kb = -1, kc = -1;
    for (int b = 0; b < 6; ++b) {
        if (G::lane_bit(PT, b) == out) kb = b;
        if (G::lane_bit(PF, b) == in) kc = b;
    }
    return kb == kc ? kb : -1;
}
template <int M, int E, int PF, int PT>
constexpr bool fperm_ok() {
#ifdef FR_FFT_NOPERM  // A/B switch: every exchange through LDS
    return false;
#else
    using G = FGeo<M, E>;
    if (PF == PT || (PF - PT != 1 && PT - PF != 1)) return false;
    for (int j = 0; j < G::e; ++j) {
        const int k = fperm_lane_bit<M, E, PF, PT>(j);
        if (k != 4 && k != 5) return false;
    }
    // every other lane bit carries the same index bit in both layouts
    for (int b = 0; b < 8; ++b) {
        bool swapped = false;
        for (int j = 0; j < G::e; ++j) swapped |= fperm_lane_bit<M, E, PF, PT>(j) == b;
        if (!swapped && G::lane_bit(PF, b) != G::lane_bit(PT, b)) return false;
    }
    return true;
#endif
}
template <int K>
__device__ __forceinline__ void fperm_swap(double& a, double& b) {
    static_assert(K == 4 || K == 5, "permlane swaps serve lane bits 4 and 5");
    const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
    const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
    unsigned lo0 = (unsigned)ua, hi0 = (unsigned)(ua >> 32), lo1 = (unsigned)ub, hi1 = (unsigned)(ub >> 32);
    if constexpr (K == 4) {
        const auto l = __builtin_amdgcn_permlane16_swap(lo0, lo1, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi0, hi1, false, false);
        lo0 = l[0], lo1 = l[1], hi0 = h[0], hi1 = h[1];
    } else {
        const auto l = __builtin_amdgcn_permlane32_swap(lo0, lo1, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi0, hi1, false, false);
        lo0 = l[0], lo1 = l[1], hi0 = h[0], hi1 = h[1];
    }
    a = __longlong_as_double((long long)(((unsigned long long)hi0 << 32) | lo0));
    b = __longlong_as_double((long long)(((unsigned long long)hi1 << 32) | lo1));
}
template <int M, int E, int PF, int PT, int j = 0>
__device__ __forceinline__ void fperm_exchange(double2 (&x)[E]) {
    constexpr int K = fperm_lane_bit<M, E, PF, PT>(j);
#pragma unroll
    for (int m = 0; m < E; ++m) {
        if (m & (1 << j)) continue;
        fperm_swap<K>(x[m].x, x[m | (1 << j)].x);
        fperm_swap<K>(x[m].y, x[m | (1 << j)].y);
    }
    if constexpr (j + 1 < FGeo<M, E>::e) fperm_exchange<M, E, PF, PT, j + 1>(x);
}

// Cross-wave exchanges that only transpose the element bits with the wave bits (lane bits
// 6, 7), position by position, with every other lane bit in place: a lane keeps the element
// whose index equals its wave bits, in the same register (forward 0 -> 1, inverse 1 -> 0 of
// k = 1), so it writes and reads E - 1 elements instead of E (FR_XKEEP).  Throughput shape
// only (XK): 512 bootstraps 2.80 -> 2.74 ms, 2048 10.66 -> 10.43 ms; the latency shape lost 3%
// to the wave-uniform branches (tools/ab_libs.sh)
#ifndef FR_XKEEP
#define FR_XKEEP 1
#endif
template <int M, int E, int PF, int PT>
constexpr bool fxkeep_ok() {
    using G = FGeo<M, E>;
    if (!FR_XKEEP || (1 << (6 + G::e)) > G::T || PF == PT) return false;
    for (int b = 0; (1 << b) < G::T; ++b) {
        if (b >= 6 && b < 6 + G::e) {
            if (G::lane_bit(PF, b) != G::lo(PT) + (b - 6) || G::lane_bit(PT, b) != G::lo(PF) + (b - 6)) return false;
        } else if (G::lane_bit(PF, b) != G::lane_bit(PT, b)) {
            return false;
        }
    }
    return true;
}
// B bootstraps per workgroup (pair shape: B = 2), bootstrap b's rows at row + b BS: one
// barrier serves the exchanges of all B
template <int M, int E, int PF, int PT, bool PRE, bool XK, int B, int BS>
__device__ __forceinline__ void fexchange(double2 (&x)[B][E], double2* row, int tl) {
    using G = FGeo<M, E>;
    if constexpr (fperm_ok<M, E, PF, PT>()) {
        // a pre-barrier would also order the next exchange's writes: keep the plan's barriers
        static_assert(!PRE, "register exchanges replace only exchanges without a pre-barrier");
#ifndef FR_FFT_NOPERMX  // timing experiment only (wrong results): register exchanges skipped
#pragma unroll
        for (int b = 0; b < B; ++b) fperm_exchange<M, E, PF, PT>(x[b]);
#endif
    } else {
#ifdef FR_FFT_NOXCHG  // timing experiment only (wrong results): LDS exchanges skipped
        return;
#endif
#ifdef FR_FFT_NOXCHG_LOCAL  // timing experiment only: wave-local LDS exchanges skipped
        if constexpr (fwave_local<M, E, PF, PT>()) return;
#endif
#ifdef FR_FFT_NOXCHG_CROSS  // timing experiment only: cross-wave LDS exchanges skipped
        if constexpr (!fwave_local<M, E, PF, PT>()) return;
#endif
        constexpr int X = PF < PT ? PF : PT;
        double2* rf = row + G::template at<X>(G::template base<PF>(tl));
        double2* rt = row + G::template at<X>(G::template base<PT>(tl));
        if constexpr (PRE) __syncthreads();
#ifdef FR_XCHG_PRIO  // A/B experiment: a wave entering an exchange issues ahead of its SIMD partner
        __builtin_amdgcn_s_setprio(FR_XCHG_PRIO);
        struct PrioReset {
            __device__ ~PrioReset() { __builtin_amdgcn_s_setprio(0); }
        } prio_reset;
#endif
        if constexpr (XK && fxkeep_ok<M, E, PF, PT>()) {  // the kept element: wave-uniform branches around its store and load
            const int q = __builtin_amdgcn_readfirstlane((tl >> 6) & (E - 1));
#pragma unroll
            for (int b = 0; b < B; ++b)
#pragma unroll
                for (int m = 0; m < E; ++m)
                    if (m != q) rf[b * BS + G::template at<X>(G::template moff<PF>(m))] = x[b][m];
            __syncthreads();
#pragma unroll
            for (int b = 0; b < B; ++b)
#pragma unroll
                for (int m = 0; m < E; ++m)
                    if (m != q) x[b][m] = rt[b * BS + G::template at<X>(G::template moff<PT>(m))];
            return;
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int m = 0; m < E; ++m) rf[b * BS + G::template at<X>(G::template moff<PF>(m))] = x[b][m];
        if constexpr (fwave_local<M, E, PF, PT>() && G::wave_top(PF)) fwave_sync();
        else __syncthreads();
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int m = 0; m < E; ++m) x[b][m] = rt[b * BS + G::template at<X>(G::template moff<PT>(m))];
    }
}
// barrier plan as in device.hip: only the first exchange of a transform and
// exchanges writing a non-wave-top layout wait before writing
template <int M, int E, int p>
constexpr bool ffwd_pre() {
    return p == 0 || !FGeo<M, E>::wave_top(p);
}
template <int M, int E, int p>
constexpr bool finv_pre() {
    return p == FGeo<M, E>::NPH - 1 || !FGeo<M, E>::wave_top(p);
}
// every LDS exchange conflict-free; register exchanges need no map, except that map XL
// also serves the MAC's last-layout accesses
template <int M, int E, int X = 0>
constexpr bool fexchanges_conflict_free() {
    using G = FGeo<M, E>;
    if constexpr (X + 1 >= G::NPH) return true;
    else
        return ((fperm_ok<M, E, X, X + 1>() && X != G::XL) || G::template b128_exchange_ok<X>()) &&
               fexchanges_conflict_free<M, E, X + 1>();
}
// NOPRE: the rows of the forward transform + MAC and of the inverse transform
// are separate buffers (latency shape).  Then no write needs a barrier before
// it: a transform's first cross-wave write follows the previous cross-wave
// exchange's barrier, which every wave reaches only after its last read of the
// other buffer; the inverse's first write (own slots) no longer meets the other
// polynomials' MAC reads.
// TWR: twiddles from the lane's registers (twr), else from the LDS table tw.
// hook(integral_constant<p>) runs after phase p's butterflies (before its exchange).
// CARRY: a pre-barrier owed by a register exchange (which writes no LDS) moves to the
// next LDS exchange's write.
// B, BS: B transforms side by side (rows b BS apart), their exchanges sharing barriers.
template <int M, int E, int p, bool NOPRE, bool TWR, int B, int BS, bool CARRY = false, class Hook>
__device__ __forceinline__ void fforward_from(double2 (&x)[B][E], double2* row, const FTwr<M, TWR ? E : 2>& twr,
                                              const double2* tw, int tl, Hook&& hook) {
#pragma unroll
    for (int b = 0; b < B; ++b) {
        if constexpr (TWR) ffwd_phase_r<M, E, p>(x[b], twr);
        else ffwd_phase<M, E, p>(x[b], tw, tl);
    }
    hook(std::integral_constant<int, p>{});
    if constexpr (p + 1 < FGeo<M, E>::NPH) {
        constexpr bool pre = !NOPRE && (ffwd_pre<M, E, p>() || CARRY), reg = fperm_ok<M, E, p, p + 1>();
        fexchange<M, E, p, p + 1, reg ? false : pre, !NOPRE, B, BS>(x, row, tl);
        fforward_from<M, E, p + 1, NOPRE, TWR, B, BS, reg && pre>(x, row, twr, tw, tl, hook);
    }
}
template <int M, int E, int p, bool NOPRE, bool TWR, int B, int BS, bool CARRY = false>
__device__ __forceinline__ void finverse_from(double2 (&x)[B][E], double2* row, const FTwr<M, TWR ? E : 2>& twr,
                                              const double2* tw, const double2* twc, int tl) {
    if constexpr (TWR && B > 1 && fradix4<M, E>() && FR_PAIR_CC) {
        // pair shape: cc = c ca recomputed per phase (20 fewer live VGPRs; the same
        // fft::cmul as ftw_load_phase, so the same bits), shared by the B transforms
        const double2 c = twr.v[3 * p], ca = twr.v[3 * p + 1];
        double2 cc;
        fft::cmul(c.x, c.y, ca.x, ca.y, cc.x, cc.y);
#pragma unroll
        for (int b = 0; b < B; ++b) cinv_r4(x[b], c, ca, cc);
    } else {
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if constexpr (TWR) finv_phase_r<M, E, p>(x[b], twr);
            else finv_phase_lds<M, E, p>(x[b], tw, twc, tl);
        }
    }
    if constexpr (p > 0) {
        constexpr bool pre = !NOPRE && (finv_pre<M, E, p>() || CARRY), reg = fperm_ok<M, E, p, p - 1>();
        fexchange<M, E, p, p - 1, reg ? false : pre, !NOPRE, B, BS>(x, row, tl);
        finverse_from<M, E, p - 1, NOPRE, TWR, B, BS, reg && pre>(x, row, twr, tw, twc, tl);
    }
}

// (K + 1) polynomials of M / E lanes each
template <int N, int K, int E>
constexpr int fbr_threads() {
    return (K + 1) * (N / 2 / E);
}
// Launch shapes (Device::launch_br_fft picks one by batch size):
//  * latency, LAT (E = 4; launches of at most one bootstrap per CU): one
//    workgroup per CU (k = 1: 8 waves; k = 2, N = 1024: 6 waves), 256 VGPRs; the
//    step's 3 x (k+1) x E Fourier GGSW slots are loaded at the top of the step
//    (they land during the digits and the forward FFT); the whole psi^k table
//    (k < 2N: no sign flips on lookup) and two sets of exchange rows (forward + MAC /
//    inverse: 3 barriers per step instead of 5) in LDS.  k = 1 keeps the lane's
//    twiddles in registers (TWR); k = 2 reads them from LDS (the 36 GGSW values
//    take the registers).
//  * pair (k = 1, B = 2; launches between the latency shape's limit and fft_pair_): the
//    latency geometry with two bootstraps per workgroup.  One set of key loads, twiddle
//    registers and barriers serves both (the two workgroups a CU would run side by side
//    in the throughput shape each load the whole key and wait at their own barriers), and
//    the two transforms give each other's exchanges independent work.  LDS: both row
//    sets per bootstrap (139 KB) + the quadrant psi table; twiddles load from global once.
//  * throughput (k = 1, E = 4: 8 waves, 128 VGPRs; E = 8: 4 waves): two workgroups per
//    CU (<= 80 KB of LDS each) hide each other's barriers and loads; a slot's
//    GGSW values are loaded one slot ahead in the MAC; psi^k from the quadrant
//    table (k < N/2) + quarter turns.  k = 2, N = 1024: E = 8 is one wave per
//    polynomial (every transform exchange wave-local), three workgroups per CU.
// LDS slot of psi^k in the monomial table.  A lane's lookup index is k = e L mod 2N
// with L = 1 + 4 brv(lane slot base), so the 16 lanes of a b128 read group share
// k mod 32 (every lookup one bank quad: ~13-way conflicts).  Folding bits 5..9 into
// the quad bits spreads them (1.8-way on average over e); a bijection on [0, 2^10)
// blocks, so it serves the N-entry and the N/2-entry (quadrant) table alike.
__device__ __forceinline__ int psi_slot(int k) { return k ^ ((k >> 6) & 15) ^ ((k >> 5) & 1); }

// Slot factor psi^(e (Lb + M sm)) = i^q psi^(e Lb), q = (e sm) mod 4 (fft::psi_quadrant of
// the base): for odd sm, q is odd exactly when the uniform e is, so the swap of an odd turn is
// one select per base shared by the slots sm = 1, 3, and every slot adds only a uniform sign
// (i^q b = i^(q-1) (i b), q - 1 even).  The same values as psi_quadrant; 11 VALU per factor
// over a lane's 4 slots instead of ~23 (latency step loop 602 -> 584 VALU per wave-step; one
// bootstrap 1.355 -> 1.324 ms, 2048 10.00 -> 9.83 ms: profiles/r03/ab_slot_factor.log).
// A 16-way uniform branch on (a_i, a_j) mod 4 that made every turn compile-time spilled
// 14-84 VGPRs in every shape and was dropped.
__device__ __forceinline__ void slot_factor(double br, double bi, uint32_t e, uint32_t sm, double& cr, double& ci) {
    const uint32_t q = (e * sm) & 3u;
    const bool swap = (sm & 1u) && (e & 1u);
    const double ar = swap ? -bi : br, ai = swap ? br : bi;
    const long long sg = (long long)((q >> 1) & 1u) << 63;
    cr = __longlong_as_double(__double_as_longlong(ar) ^ sg);
    ci = __longlong_as_double(__double_as_longlong(ai) ^ sg);
}
// twiddles in registers (latency shape, k = 1)
template <int K, bool LAT>
constexpr bool fbr_twr() {
    return LAT && K == 1 && FR_LAT_TWR;
}
// radix-4 inverse with LDS twiddles: the product table c ca (M/2 entries, indexed like c)
template <int N, int K, int E, bool LAT>
constexpr int fbr_twc_entries() {
    return fradix4<N / 2, E>() && !fbr_twr<K, LAT>() ? N / 4 : 0;
}
// LDS of a shape with B bootstraps per workgroup.  The pair shape (B = 2) keeps the
// latency shape's two row sets per bootstrap (139 KB at k = 1) by dropping the forward
// twiddle table (its registers load from global memory once) and using the quadrant
// psi table; its multi-value terms live in the inverse rows after the loop.
template <int N, int K, int E, bool LAT, int B = 1>
constexpr size_t fbr_smem_bytes() {
    return 16 * ((LAT ? 2 : 1) * B * (K + 1) * (size_t)FGeo<N / 2, E>::NP + (B == 1 ? (size_t)N / 2 : 0) +
                 (LAT && B == 1 ? 2 * (size_t)N : (size_t)N / 2) + (size_t)fbr_twc_entries<N, K, E, LAT>()) +
           B * (16 * MAX_OUT + 2 * 1026) + (B == 1 ? 4 * 17 * MAX_OUT : 0) + 2 * 514;
}
// workgroups per CU of the throughput shapes (LDS: fbr_smem_bytes * this <= 160 KB)
template <int K, int E>
constexpr int fbr_tp_groups() {
    return K == 1 ? 2 : (E == 8 ? 3 : 2);
}
// waves per SIMD the register allocation must allow
template <int N, int K, int E, bool LAT>
constexpr int fbr_min_waves() {
    if (LAT) return E == 2 ? 4 : 2;  // E = 2 (FR_LAT_E2 experiment): 16 waves, 4 per SIMD
    if (K == 1) return E == 4 ? 4 : 2;
    return E == 4 ? 3 : 2;  // k = 2: 2 x 6 waves (E = 4); E = 8: the one-slot-ahead loads need > 168 VGPRs
}
// Fourier-key loads: buffer loads with the key's resource in SGPRs, the uniform part
// of the offset (step, GGSW, row, slot) in soffset and the lane's byte offset as the
// only VGPR operand, so a load costs no VALU address arithmetic (gfx950 raw buffer
// resource: word 3 = 0x00020000; the key is < 2 GiB)
typedef unsigned int fr_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bsk_rsrc(const double2* bsk) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)bsk, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double2 bsk_load(__amdgpu_buffer_rsrc_t r, uint32_t lane_off, uint32_t uoff) {
    const fr_v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)lane_off, (int)uoff, 0);
    double2 d;
    __builtin_memcpy(&d, &v, 16);
    return d;
}

// row r != P of the MAC: the q-th other polynomial in ascending order
template <int K>
__device__ __forceinline__ int other_row(int P, int q) {
    return q < P ? q : q + 1;
}
// the 3 (K+1) Fourier GGSW values of slot m for this lane: [g][own row, other rows...]
// (Fourier GGSW [r][c][m][lane]: row r, output column c = P; sbase: the step's byte offset)
template <int M, int T, int K>
__device__ __forceinline__ void load_slot(double2 (&B)[3][K + 1], __amdgpu_buffer_rsrc_t rs, uint32_t sbase, int P,
                                          int m, uint32_t lane_off) {
    constexpr uint32_t GG = (uint32_t)(K + 1) * (K + 1) * M;
#pragma unroll
    for (int gg = 0; gg < 3; ++gg) {
        B[gg][0] = bsk_load(rs, lane_off, sbase + 16u * (gg * GG + (uint32_t)(P * (K + 1) + P) * M + (uint32_t)m * T));
#pragma unroll
        for (int q = 0; q < K; ++q)
            B[gg][1 + q] = bsk_load(
                rs, lane_off, sbase + 16u * (gg * GG + (uint32_t)(other_row<K>(P, q) * (K + 1) + P) * M + (uint32_t)m * T));
    }
}

// value of the test polynomial at position t < N: the LUT polynomial (box N/16,
// recentred by half a box, -f(0) in the last half box) or (Delta/2) * sum X^j
template <int N>
__device__ __forceinline__ uint64_t test_poly(int t, bool direct, const uint8_t* lut0) {
    constexpr int box = N / 16, half = box / 2;
    if (!direct) return 1ULL << (DELTA_LOG - 1);
    const int mm = (t + half) / box;
    return mm < 16 ? (uint64_t)lut0[mm] << DELTA_LOG : (uint64_t)0 - ((uint64_t)lut0[0] << DELTA_LOG);
}
// sum_t d_t (X^pos_t A)[j] mod 2^64 (multi-value w-step, terms as device.hip)
template <int N>
__device__ __forceinline__ uint64_t w_step64(const uint64_t* row, const uint32_t* terms, int nt, int j) {
    uint64_t acc = 0;
    for (int t = 0; t < nt; ++t) {
        const uint32_t tm = terms[t];
        int src = j - (int)(tm & 0xFFFF);
        int64_t d = (int64_t)(tm >> 16) - 128;
        if (src < 0) {
            src += N;
            d = -d;
        }
        acc += (uint64_t)d * row[src];
    }
    return acc;
}

template <int N, int K, int E, bool LAT, int B = 1>
__global__ void __launch_bounds__((fbr_threads<N, K, E>()), (fbr_min_waves<N, K, E, LAT>()))
k_blind_rotate_fft(const uint64_t* __restrict__ ks, int ks_stride, int n, const DevGate* __restrict__ gates,
                   int n_gates, const double2* __restrict__ bsk, const double2* __restrict__ tw_g,
                   const double2* __restrict__ psi_g, const uint16_t* __restrict__ leaf_g, uint64_t* __restrict__ arena,
                   int slot_stride) {
    constexpr int M = N / 2;
    using G = FGeo<M, E>;
    static_assert(fexchanges_conflict_free<M, E>(), "LDS maps must make every exchange conflict-free");
    static_assert(!LAT || E == 4 || E == 2, "the latency shape holds a step's GGSW values in registers: E = 4 (2: experiment)");
    static_assert(B == 1 || (B == 2 && LAT && K == 1 && E == 4), "pair shape: the k = 1 latency geometry");
    constexpr int NB = E >= 4 ? E / 4 : 1;  // psi bases per lane (slots m >> 2 share one)
    constexpr int T = M / E, NT = (K + 1) * T, LAST = G::NPH - 1, XL = G::XL;
    constexpr int LOG2N2 = G::LOG + 2;  // log2(2N)
    constexpr bool TWR = fbr_twr<K, LAT>();  // twiddles in registers
    constexpr int BS = (K + 1) * G::NP;      // one bootstrap's exchange rows
    constexpr bool PSIQ = !LAT || B > 1;     // psi^k from the quadrant table (k < N/2) + quarter turns
    extern __shared__ __attribute__((aligned(16))) double2 fsm[];
    double2* xbuf = fsm;                  // B x (K+1) rows of NP complex: bootstrap b, row P at b BS + P NP
    double2* ibuf = LAT ? xbuf + B * BS : xbuf;  // inverse-transform rows (latency shapes: separate)
    double2* tw = xbuf + (LAT ? 2 : 1) * B * BS;  // M forward twiddles (B = 1)
    constexpr int NPSI = PSIQ ? N / 2 : 2 * N;  // (latency shape: the whole circle, no sign flips)
    double2* psi = tw + (B == 1 ? M : 0);  // psi^k, k < NPSI
    double2* twc = psi + NPSI;            // radix-4 products c ca (fbr_twc_entries)
    constexpr int NTWC = fbr_twc_entries<N, K, E, LAT>();
    uint8_t* lut = (uint8_t*)(twc + NTWC);                 // [B][16 * MAX_OUT]
    uint16_t* abar = (uint16_t*)(lut + B * 16 * MAX_OUT);  // [B][1026]: n (<= 1024), zero-padded to even
    uint32_t* wterms = B == 1 ? (uint32_t*)(abar + 1026) : (uint32_t*)ibuf;  // multi-value terms, [B][16 MAX_OUT]
    int* wcnt = (int*)(wterms + B * 16 * MAX_OUT);                           // [B][MAX_OUT]
    uint16_t* nxt = B == 1 ? (uint16_t*)(wcnt + MAX_OUT) : abar + B * 1026;  // (latency shapes) next unskipped step

    const int tid = threadIdx.x;
    const int P = __builtin_amdgcn_readfirstlane(tid / T), tl = tid % T;  // wave-uniform polynomial
    // bootstrap b of this workgroup: gate B blockIdx + b (an odd count's last pair repeats its
    // gate and writes it once)
    int gb[B];
    bool has[B];
    const uint64_t* in[B];
    int n_out[B], kind[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int gi = B * (int)blockIdx.x + b;
        has[b] = gi < n_gates;
        gb[b] = has[b] ? gi : B * (int)blockIdx.x;
        in[b] = ks + (size_t)gb[b] * ks_stride;
        n_out[b] = gates[gb[b]].n_out;
        kind[b] = gates[gb[b]].direct;
    }
    if constexpr (B == 1)
        for (int i = tid; i < M; i += NT) tw[i] = tw_g[i];
    for (int i = tid; i < NPSI; i += NT) psi[psi_slot(i)] = psi_g[i];
    // twc[2^s0 + b] = tw[2^s0 + b] * tw[2^(s0+1) + 2b] for even s0 (fft::cmul, as the oracle)
    for (int i = 1 + tid; i < NTWC; i += NT) {
        const int s0 = 31 - __builtin_clz((unsigned)i), b = i - (1 << s0);
        if (s0 & 1) continue;
        const double2 c = tw_g[i], ca = tw_g[(2 << s0) + 2 * b];
        fft::cmul(c.x, c.y, ca.x, ca.y, twc[i].x, twc[i].y);
    }
    uint32_t bbar[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        uint8_t* lb = lut + b * 16 * MAX_OUT;
        uint16_t* ab = abar + b * 1026;
        for (int i = tid; i < 16 * n_out[b]; i += NT) lb[i] = gates[gb[b]].lut[i / 16][i % 16];
        for (int i = tid; i < n; i += NT) ab[i] = (uint16_t)mod_switch(in[b][i], LOG2N2);
        if (tid == 0) ab[n] = 0;  // pad an odd n
        bbar[b] = mod_switch(in[b][n], LOG2N2);
    }
    // leaf exponents mod M of this lane's slot bases (slots 4b): L(j) = 1 + 4 brv(j)
    // (fft::Tables::leaf, checked against the table in tests/test_fft.py)
    uint32_t Lb[NB];
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
        Lb[bb] = (1u + 4u * (__brev((uint32_t)G::template idx<LAST>(tl, 4 * bb)) >> (32 - G::LOG))) & (uint32_t)(M - 1);
    __syncthreads();

    // accumulator (f64 torus, fft.h), natural order: lane holds coefficients j and
    // j + M for j = idx<0>(tl, m); mask polynomials 0, body (polynomial K) X^-bbar * V
    double alo[B][E], ahi[B][E];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const bool direct = kind[b] == JOB_DIRECT;
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int j = G::template idx<0>(tl, m);
            uint64_t v[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int s = (j + h * M + (int)bbar[b]) & (2 * N - 1);
                const uint64_t tv = test_poly<N>(s & (N - 1), direct, lut + b * 16 * MAX_OUT);
                v[h] = s < N ? tv : (uint64_t)0 - tv;
            }
            alo[b][m] = P == K ? fft::acc_of_torus(v[0]) : 0.0;
            ahi[b][m] = P == K ? fft::acc_of_torus(v[1]) : 0.0;
        }
    }

    double2* row = xbuf + P * G::NP;
    double2* irow = ibuf + P * G::NP;
    const int bl = G::template base<LAST>(tl);
    double2* row_bl = row + G::template at<XL>(bl);
    const double2* orow_bl[K];  // the other polynomials' rows, ascending
#pragma unroll
    for (int q = 0; q < K; ++q) orow_bl[q] = xbuf + other_row<K>(P, q) * G::NP + G::template at<XL>(bl);
    constexpr uint32_t GG = (uint32_t)(K + 1) * (K + 1) * M;  // complex values per Fourier GGSW: [r][c][m][lane]
    const __amdgpu_buffer_rsrc_t rs = bsk_rsrc(bsk);
    const uint32_t lane_off = 16u * (uint32_t)tl;
    const int steps = (n + 1) / 2;
    // latency shape: Fourier GGSW slots of a step for this lane, [g][own, other rows][m],
    // and (k = 1) the lane's twiddles
    double2 gv[3][K + 1][LAT ? E : 1];
    FTwr<M, TWR ? E : 2> twr;
    if constexpr (TWR) ftw_load_phase<M, E, 0, B == 1 ? FR_TW_SGPR_LAT : FR_TW_SGPR_PAIR>(twr, B == 1 ? tw : tw_g, tl);
#ifdef FR_BR_TIMING
    uint64_t tseg[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tlast = __builtin_amdgcn_s_memtime();
    const uint64_t tstart = tlast;
#endif
    // latency shape: GGSW g's slots of step tt for this lane ([g][own, other rows][m])
    auto load_ggsw = [&](int gg, int tt) {
        const uint32_t sb = (uint32_t)__builtin_amdgcn_readfirstlane(tt) * (3u * GG * 16u);
#pragma unroll
        for (int m = 0; m < E; ++m) {
#ifdef FR_FFT_NOBSK  // timing experiment only (wrong results): no GGSW traffic
#pragma unroll
            for (int r = 0; r <= K; ++r) gv[gg][r][m] = make_double2(tt + gg + r, m);
#else
            gv[gg][0][m] =
                bsk_load(rs, lane_off, sb + 16u * (gg * GG + (uint32_t)(P * (K + 1) + P) * M + (uint32_t)m * T));
#pragma unroll
            for (int q = 0; q < K; ++q)
                gv[gg][1 + q][m] = bsk_load(
                    rs, lane_off,
                    sb + 16u * (gg * GG + (uint32_t)(other_row<K>(P, q) * (K + 1) + P) * M + (uint32_t)m * T));
#endif
        }
    };
    // latency shape, LATPF: groups 0 .. NPF-1 of a step's key values are loaded one
    // step ahead -- right after the previous step's MAC, when their registers are dead --
    // so that they have the inverse FFT, the accumulate and the forward FFT to land (a
    // single CU streams ~50 GB/s of key at 3.9 us per step); the others across the
    // step's own forward FFT.  The next unskipped step comes from the table nxt (no
    // control flow around the prefetch, which keeps it after the MAC's last use).
    constexpr int NPF = LAT ? (B > 1 ? FR_PAIR_PF : K == 1 ? FR_LAT_PF : FR_LAT_PF2) : 0;
    constexpr bool LATPF = NPF > 0;
    // step t is skipped when every bootstrap's pair is (0, 0): X^0 acc - acc = 0.  The pair
    // shape runs a step that is zero for one bootstrap only: its factors c - 1 are exact
    // zeros, so its MAC output is 0 and the accumulate adds +-0.
    auto idle = [&](int t) {
        uint32_t z = 0;
#pragma unroll
        for (int b = 0; b < B; ++b) z |= abar[b * 1026 + 2 * t] | abar[b * 1026 + 2 * t + 1];
        return z == 0;
    };
    if constexpr (LATPF) {
        for (int t = tid; t <= steps; t += NT) {
            int tt = t;
            while (tt < steps && idle(tt)) ++tt;
            nxt[t] = (uint16_t)tt;
        }
        __syncthreads();
        const int t0 = __builtin_amdgcn_readfirstlane((int)nxt[0]);
        for (int gg = 0; gg < NPF; ++gg) load_ggsw(gg, t0 < steps ? t0 : 0);
    }
#if defined(FR_PRIO_HALF_LAT) || defined(FR_PRIO_HALF_PAIR)
    // A/B experiment (MI355X_MICROARCH.md "Two waves per SIMD", item 4): the second half of an
    // 8-wave workgroup (waves 4-7: polynomial 1) loses VALU arbitration to its older SIMD
    // partner at every segment head; one static s_setprio for that half before the loop
    if constexpr (LAT) {
#ifdef FR_PRIO_HALF_LAT
        if (B == 1 && tid >= NT / 2) __builtin_amdgcn_s_setprio(FR_PRIO_HALF_LAT);
#endif
#ifdef FR_PRIO_HALF_PAIR
        if (B == 2 && tid >= NT / 2) __builtin_amdgcn_s_setprio(FR_PRIO_HALF_PAIR);
#endif
    }
#endif
    for (int t = 0; t < steps; ++t) {
        if (idle(t)) continue;  // (uniform branch)
        FBR_STAMP(0);
        // the step's byte offset in the key (uniform: soffset of every load)
        const uint32_t sbase = (uint32_t)__builtin_amdgcn_readfirstlane(t) * (3u * GG * 16u);
        // groups NPF.. of this step: G_TOP at the top of the step, G_L1 / G_L2 after forward
        // phases FR_LAT_LOAD1 / FR_LAT_LOAD2 (3: none).  k = 1, NPF = 2: the third group at the
        // top (tools/ab_libs.sh: 1.34 ms; after forward phase 0 / 2 / 3: 1.33 / 1.38 / 1.38 ms;
        // after the previous inverse: 1.35 ms); k = 2 keeps it after phase 3 (1.67 vs 1.71 ms)
        // The pair shape (NPF = 1) loads its second group after forward phase FR_PAIR_LOAD and
        // its third after FR_PAIR_LOAD2 = 4, right before the MAC barrier (the pair's 64 live
        // transform values leave no room for a group across the whole transform).
        constexpr int G_TOP = !LAT || B > 1 ? 3 : (NPF < 2 || K == 1) ? NPF : 3;
        constexpr int G_L1 = !LAT ? 3 : B > 1 ? NPF : G_TOP + 1 < 3 ? G_TOP + 1 : 3;
        constexpr int G_L2 = !LAT ? 3 : B > 1 ? (NPF + 1 < 3 ? NPF + 1 : 3) : G_TOP == 3 ? NPF : G_TOP + 2 < 3 ? G_TOP + 2 : 3;
        constexpr int PH_L1 = B > 1 ? FR_PAIR_LOAD : FR_LAT_LOAD1;
        constexpr int PH_L2 = B > 1 ? FR_PAIR_LOAD2 : FR_LAT_LOAD2;
        // a group loaded after a forward phase needs that phase to exist: an out-of-range
        // -D knob would skip the load and leave the MAC reading stale key registers
        static_assert(G_L1 >= 3 || PH_L1 < G::NPH, "FR_PAIR_LOAD / FR_LAT_LOAD1 past the last forward phase");
        static_assert(G_L2 >= 3 || PH_L2 < G::NPH, "FR_PAIR_LOAD2 / FR_LAT_LOAD2 past the last forward phase");
        if constexpr (G_TOP < 3) {
            __builtin_amdgcn_sched_barrier(0);
            load_ggsw(G_TOP, t);
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t ei[B], ej[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            ei[b] = __builtin_amdgcn_readfirstlane((uint32_t)abar[b * 1026 + 2 * t]);
            ej[b] = __builtin_amdgcn_readfirstlane((uint32_t)abar[b * 1026 + 2 * t + 1]);
        }
        double bre[B][2][NB], bim[B][2][NB];
        auto psi_factors = [&]() {
#pragma unroll
            for (int b = 0; b < B; ++b)
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) {
                        const uint32_t k = __umul24(h == 0 ? ei[b] : ej[b], Lb[bb]) & (2 * N - 1);
                        if constexpr (!PSIQ) {  // psi^k, k < 2N, straight from the table
#ifdef FR_FFT_NOPSI  // timing experiment only (wrong results): no table lookups
                            const double2 c = make_double2((double)k, 0.5);
#else
                            const double2 c = psi[psi_slot((int)k)];
#endif
                            bre[b][h][bb] = c.x;
                            bim[b][h][bb] = c.y;
                        } else {
                            const double2 q = psi[psi_slot((int)(k & (N / 2 - 1)))];
                            fft::psi_quadrant(q.x, q.y, k >> (LOG2N2 - 2), bre[b][h][bb], bim[b][h][bb]);
                        }
                    }
        };
        if constexpr (LAT && B == 1) psi_factors();
        // 1. signed gadget digits, folded: x = d_j + i d_(j+M)
        double2 x[B][E];
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int m = 0; m < E; ++m)
                x[b][m] = make_double2(fft::acc_digit<23>(alo[b][m]), fft::acc_digit<23>(ahi[b][m]));
        FBR_STAMP(1);
        // 2. forward FFT (latency shape: GGSW groups 1 and 2 issued at phase boundaries)
        fforward_from<M, E, 0, LAT, TWR, B, BS>(x, row, twr, tw, tl, [&](auto ph) {
            if constexpr (LAT) {
                constexpr int p = decltype(ph)::value;
                if constexpr (p == PH_L1 && G_L1 < 3) {
                    __builtin_amdgcn_sched_barrier(0);
                    load_ggsw(G_L1, t);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if constexpr (p == PH_L2 && G_L2 < 3) {
                    __builtin_amdgcn_sched_barrier(0);
                    load_ggsw(G_L2, t);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        });
        FBR_STAMP(2);
        // 3. MAC with the three GGSWs of the pair and their monomial factors
#ifndef FR_FFT_NOMACX  // timing experiment only (wrong results): no MAC exchange
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int m = 0; m < E; ++m) row_bl[b * BS + G::template at<XL>(G::template moff<LAST>(m))] = x[b][m];
#endif
        // FR_MAC_EARLY (latency shape): everything of the MAC that does not read the other
        // polynomials -- slot factors, the key-only K_r and the own-row product D_P K_P -- runs
        // between the row writes and the barrier (the writes' completion hides behind it), the
        // key registers die there, so the next step's prefetch issues before the barrier too
        // (its issue cost in the barrier's wait); after the barrier only the other rows' reads
        // and one cmac each.  Every value's operation sequence is the one below: same bits.
        constexpr bool MAC_EARLY = LAT && B == 1 && FR_MAC_EARLY;
        if constexpr (MAC_EARLY) {
            double kxr_e[E][K], kxi_e[E][K];
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const double2 own = x[0][m];
                const uint32_t sm = ((m & 1) << 1) | ((m >> 1) & 1);  // brv2(m & 3)
                double cr[3], ci[3];
#pragma unroll
                for (int h = 1; h < 3; ++h)
                    slot_factor(bre[0][h - 1][m >> 2], bim[0][h - 1][m >> 2], h == 1 ? ei[0] : ej[0], sm, cr[h], ci[h]);
                fft::cmul(cr[1], ci[1], cr[2], ci[2], cr[0], ci[0]);
                double kor, koi;
#pragma unroll
                for (int gg = 0; gg < 3; ++gg) {
                    const double c1r = cr[gg] - 1.0, c1i = ci[gg];
                    const double2 Bo = gv[gg][0][m];
                    if (gg == 0) fft::cmul(Bo.x, Bo.y, c1r, c1i, kor, koi);
                    else fft::cmac(Bo.x, Bo.y, c1r, c1i, kor, koi);
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        const double2 Bx = gv[gg][1 + q][m];
                        if (gg == 0) fft::cmul(Bx.x, Bx.y, c1r, c1i, kxr_e[m][q], kxi_e[m][q]);
                        else fft::cmac(Bx.x, Bx.y, c1r, c1i, kxr_e[m][q], kxi_e[m][q]);
                    }
                }
                double zr, zi;
                fft::cmul(own.x, own.y, kor, koi, zr, zi);
                x[0][m] = make_double2(zr, zi);
            }
            if constexpr (LATPF && FR_MAC_EARLY == 1) {  // the next step's key, into the registers just freed
                const int tn = __builtin_amdgcn_readfirstlane((int)nxt[t + 1]);
                __builtin_amdgcn_sched_barrier(0);
                for (int gg = 0; gg < NPF; ++gg) load_ggsw(gg, tn < steps ? tn : t);
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
#pragma unroll
            for (int m = 0; m < E; ++m) {
                double zr = x[0][m].x, zi = x[0][m].y;
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    const double2 oth = orow_bl[q][G::template at<XL>(G::template moff<LAST>(m))];
                    fft::cmac(oth.x, oth.y, kxr_e[m][q], kxi_e[m][q], zr, zi);
                }
                x[0][m] = make_double2(zr, zi);
            }
            if constexpr (LATPF && FR_MAC_EARLY == 2) {  // (2: the prefetch after the cross terms, as without)
                const int tn = __builtin_amdgcn_readfirstlane((int)nxt[t + 1]);
                __builtin_amdgcn_sched_barrier(0);
                for (int gg = 0; gg < NPF; ++gg) load_ggsw(gg, tn < steps ? tn : t);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
        // throughput shapes: slot m's GGSW values, loaded one slot ahead (E = 8) or
        // at the top of the slot (E = 4, 128 VGPRs: the other workgroup hides the wait)
        constexpr bool AHEAD = !LAT && E == 8;
#ifdef FR_TP_NOPRE0  // A/B switch: E = 4 throughput shape loads slot 0 in-slot too
        constexpr bool PRE0 = AHEAD;
#else
        constexpr bool PRE0 = !LAT;  // slot 0 lands during the MAC barrier and row exchange
#endif
        double2 Bc[3][K + 1];
        if constexpr (PRE0) load_slot<M, T, K>(Bc, rs, sbase, P, 0, lane_off);
#ifndef FR_FFT_NOMACX
        __syncthreads();
#endif
        // slot factors psi^(e L) for e = a_i, a_j and their product for a_i + a_j.
        // Slot m of this lane has L = Lb + M s_m: Lb = L mod M is shared by the
        // slots of equal m >> 2 (E/4 bases per lane) and s_m = brv2(m & 3) (fft.h: L(j) =
        // 1 + 4 brv(j)).  psi^(M s e) = i^(s e) is an exact quarter turn (the table
        // itself is quadrant-reduced), so one lookup per (e, base) serves every slot.
        // latency shape: computed at the top of the step (the lookups' LDS latency hides
        // behind the digits and the forward FFT); throughput shapes: here (VGPR budget)
        if constexpr (!LAT || B > 1) psi_factors();
#pragma unroll
        for (int m = 0; m < E; ++m) {
            double2 Bn[3][K + 1];
            if constexpr (AHEAD) {
                if (m + 1 < E) load_slot<M, T, K>(Bn, rs, sbase, P, m + 1, lane_off);
                __builtin_amdgcn_sched_barrier(0);
            } else if constexpr (!LAT) {
                if (!PRE0 || m > 0) load_slot<M, T, K>(Bc, rs, sbase, P, m, lane_off);
            }
#pragma unroll
            for (int b = 0; b < B; ++b) {  // (the pair shape: both bootstraps on one set of key values)
                const double2 own = x[b][m];
                double2 oth[K];
#pragma unroll
#ifdef FR_FFT_NOMACX
                for (int q = 0; q < K; ++q) oth[q] = make_double2(own.y, own.x);
#else
                for (int q = 0; q < K; ++q) oth[q] = orow_bl[q][b * BS + G::template at<XL>(G::template moff<LAST>(m))];
#endif
                const uint32_t sm = ((m & 1) << 1) | ((m >> 1) & 1);  // brv2(m & 3)
                double cr[3], ci[3];
#pragma unroll
                for (int h = 1; h < 3; ++h)  // uniform quarter turn
                    slot_factor(bre[b][h - 1][m >> 2], bim[b][h - 1][m >> 2], h == 1 ? ei[b] : ej[b], sm, cr[h], ci[h]);
#ifdef FR_FFT_NOC0  // timing experiment only (wrong results): no pair-monomial product
                cr[0] = cr[1] + cr[2], ci[0] = ci[1];
#else
                fft::cmul(cr[1], ci[1], cr[2], ci[2], cr[0], ci[0]);
#endif
                // per row r: K_r = sum_g B_g[r][P] (c_g - 1), g ascending; then
                // z = D_P K_P + sum_(r != P, ascending) D_r K_r  (own row first).
                // 16 (K + 1) VALU per slot (k = 1: 32, against 36 for sum_g (c_g - 1) y_g)
                double kor, koi, kxr[K], kxi[K];
#pragma unroll
                for (int gg = 0; gg < 3; ++gg) {
                    const double c1r = cr[gg] - 1.0, c1i = ci[gg];
                    const double2 Bo = LAT ? gv[gg][0][LAT ? m : 0] : Bc[gg][0];
                    if (gg == 0) fft::cmul(Bo.x, Bo.y, c1r, c1i, kor, koi);
                    else fft::cmac(Bo.x, Bo.y, c1r, c1i, kor, koi);
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        const double2 Bx = LAT ? gv[gg][1 + q][LAT ? m : 0] : Bc[gg][1 + q];
                        if (gg == 0) fft::cmul(Bx.x, Bx.y, c1r, c1i, kxr[q], kxi[q]);
                        else fft::cmac(Bx.x, Bx.y, c1r, c1i, kxr[q], kxi[q]);
                    }
                }
                double zr, zi;
                fft::cmul(own.x, own.y, kor, koi, zr, zi);
#pragma unroll
                for (int q = 0; q < K; ++q) fft::cmac(oth[q].x, oth[q].y, kxr[q], kxi[q], zr, zi);
                x[b][m] = make_double2(zr, zi);
            }
            if constexpr (!LAT) {
                // keep the loads one slot ahead / in their slot, not all hoisted
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (AHEAD) {
#pragma unroll
                for (int gg = 0; gg < 3; ++gg)
#pragma unroll
                    for (int r = 0; r <= K; ++r) Bc[gg][r] = Bn[gg][r];
            }
        }
        if constexpr (LATPF) {  // the next step's key, into the registers the MAC just freed
            const int tn = __builtin_amdgcn_readfirstlane((int)nxt[t + 1]);
            __builtin_amdgcn_sched_barrier(0);
            for (int gg = 0; gg < NPF; ++gg) load_ggsw(gg, tn < steps ? tn : t);
            __builtin_amdgcn_sched_barrier(0);
        }
        }  // !MAC_EARLY
        FBR_STAMP(3);
        // 4. inverse FFT (times M; 1/M is in the key), accumulate, reduce mod 2^64
        finverse_from<M, E, LAST, LAT, TWR, B, BS>(x, irow, twr, tw, twc, tl);
        FBR_STAMP(4);
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                alo[b][m] = fft::acc_reduce<23>(alo[b][m] + x[b][m].x);
                ahi[b][m] = fft::acc_reduce<23>(ahi[b][m] + x[b][m].y);
            }
        FBR_STAMP(5);
    }
#ifdef FR_BR_TIMING
    if (blockIdx.x == 0 && tid == 0)
        printf("FBR_TIMING E=%d LAT=%d steps=%d total=%lu digits=%lu fwd=%lu mac=%lu inv=%lu acc=%lu top=%lu\n", E, (int)LAT,
               steps, (unsigned long)(__builtin_amdgcn_s_memtime() - tstart), (unsigned long)tseg[1],
               (unsigned long)tseg[2], (unsigned long)tseg[3], (unsigned long)tseg[4], (unsigned long)tseg[5],
               (unsigned long)tseg[0]);
#endif

    // publish the accumulator as u64 [P][N] over the exchange rows
    // (pair shape: bootstrap b's u64 rows at b (K+1) N, inside the forward rows; its terms in
    // the inverse rows)
    __syncthreads();
    uint64_t* accs = (uint64_t*)xbuf;
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int j = G::template idx<0>(tl, m);
            accs[(b * (K + 1) + P) * N + j] = fft::torus_of_acc(alo[b][m]);
            accs[(b * (K + 1) + P) * N + j + M] = fft::torus_of_acc(ahi[b][m]);
        }
    static_assert(B == 1 || 8 * B * (K + 1) * N <= 16 * B * BS, "pair shape: u64 rows inside the forward rows");
#pragma unroll
    for (int b = 0; b < B; ++b)
        if (tid < n_out[b] && kind[b] == JOB_MULTI) {
            // multi-value terms (device.hip lut_terms)
            constexpr int box = N / 16, half = box / 2;
            const uint8_t* lf = lut + b * 16 * MAX_OUT + 16 * tid;
            uint32_t* terms = wterms + b * 16 * MAX_OUT + 16 * tid;
            int nt = 0;
            for (int tt = 1; tt <= 16; ++tt) {
                const int d = tt < 16 ? (int)lf[tt] - (int)lf[tt - 1] : -((int)lf[0] + (int)lf[15]);
                if (d != 0) terms[nt++] = (uint32_t)(tt < 16 ? tt * box - half : N - half) | ((uint32_t)(d + 128) << 16);
            }
            wcnt[b * MAX_OUT + tid] = nt;
        }
    __syncthreads();
    constexpr int big = K * N;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        if (!has[b]) continue;
        const uint64_t* ab = accs + b * (K + 1) * N;
        if (kind[b] != JOB_MULTI) {
            uint64_t* out = arena + (size_t)gates[gb[b]].out_slot[0] * slot_stride;
            const uint64_t post = kind[b] == JOB_SIGN ? (1ULL << (DELTA_LOG - 1)) : 0;
            for (int c = tid; c <= big; c += NT) {
                const int pp = c < big ? c / N : K, t = c < big ? c % N : 0;
                const int j = t == 0 ? 0 : N - t;
                const uint64_t v = ab[pp * N + j];
                out[c] = (t != 0 ? (uint64_t)0 - v : v) + (c == big ? post : 0);
            }
            continue;
        }
        for (int f = 0; f < n_out[b]; ++f) {
            const uint32_t* tf = wterms + b * 16 * MAX_OUT + 16 * f;
            const int nt = wcnt[b * MAX_OUT + f];
            uint64_t* out = arena + (size_t)gates[gb[b]].out_slot[f] * slot_stride;
            for (int c = tid; c <= big; c += NT) {
                const int pp = c < big ? c / N : K, t = c < big ? c % N : 0;
                const int j = t == 0 ? 0 : N - t;
                const uint64_t v = w_step64<N>(ab + pp * N, tf, nt, j);
                out[c] = t != 0 ? (uint64_t)0 - v : v;
            }
        }
    }
}

// The pair shape's one instantiation is compiled in its own translation unit,
// fft_br_pair.hip, under the max-ILP machine scheduler (Makefile: PAIR_SCHED).  A/B on one box
// (profiles/r06/ab_sched.log): 512 / 2048 bootstraps 1.6% / 1.4% faster, while the latency shape
// loses 6% under that scheduler and keeps the default here.  Scheduling does not change an
// operation, so the results are the same bits.
#ifndef FR_BR_PAIR_TU
extern template __global__ void k_blind_rotate_fft<2048, 1, 4, true, 2>(const uint64_t*, int, int, const DevGate*, int,
                                                                         const double2*, const double2*, const double2*,
                                                                         const uint16_t*, uint64_t*, int);
#endif

// Dual shape (round 4 experiment, k = 1, FR_FFT_DUAL=1): one bootstrap per workgroup on
// M / E = 256 lanes (4 waves), each lane holding the same slots of BOTH polynomials
// (x[P][E]: the pair shape's B dimension carries the polynomial), two workgroups per CU.
// Both digit polynomials of a slot are in the lane, so the MAC needs no exchange and no
// barrier: the lane computes both output columns from all four (r, c) key values of its
// slots (the same operation sequence per output as the other shapes: bit-identical).  The
// forward and inverse share one row set (pre-barriers, as the throughput shape: 4 barriers
// per step), 54 KB of LDS per workgroup.  Each workgroup streams the whole key (the pair
// shape shares it between two bootstraps); the two workgroups of a CU have their own
// barriers, so one computes while the other waits.
template <int N>
constexpr size_t fbr_dual_smem_bytes() {
    return 16 * (2 * (size_t)FGeo<N / 2, 4>::NP + (size_t)N / 2) + 16 * MAX_OUT + 2 * 1026 + 4 * 16 * MAX_OUT +
           4 * MAX_OUT;
}
template <int N>
__global__ void __launch_bounds__(N / 8, 2)
k_blind_rotate_fft_dual(const uint64_t* __restrict__ ks, int ks_stride, int n, const DevGate* __restrict__ gates,
                        int n_gates, const double2* __restrict__ bsk, const double2* __restrict__ tw_g,
                        const double2* __restrict__ psi_g, const uint16_t* __restrict__ leaf_g,
                        uint64_t* __restrict__ arena, int slot_stride) {
    constexpr int K = 1, E = 4, M = N / 2, B = 2;
    using G = FGeo<M, E>;
    static_assert(fexchanges_conflict_free<M, E>(), "LDS maps must make every exchange conflict-free");
    static_assert(fradix4<M, E>(), "dual shape: the k = 1 geometry (radix-4 inverse)");
    constexpr int T = M / E, NT = T, LAST = G::NPH - 1;
    constexpr int LOG2N2 = G::LOG + 2;
    constexpr int BS = G::NP;  // polynomial P's exchange row at P BS
    extern __shared__ __attribute__((aligned(16))) double2 fsm[];
    double2* xbuf = fsm;
    double2* psi = xbuf + B * BS;  // quadrant table psi^k, k < N/2
    uint8_t* lut = (uint8_t*)(psi + N / 2);
    uint16_t* abar = (uint16_t*)(lut + 16 * MAX_OUT);
    uint32_t* wterms = (uint32_t*)(abar + 1026);
    int* wcnt = (int*)(wterms + 16 * MAX_OUT);

    const int tl = threadIdx.x;
    const int gi = (int)blockIdx.x;
    const uint64_t* in = ks + (size_t)gi * ks_stride;
    const int n_out = gates[gi].n_out, kind = gates[gi].direct;
    for (int i = tl; i < N / 2; i += NT) psi[psi_slot(i)] = psi_g[i];
    for (int i = tl; i < 16 * n_out; i += NT) lut[i] = gates[gi].lut[i / 16][i % 16];
    for (int i = tl; i < n; i += NT) abar[i] = (uint16_t)mod_switch(in[i], LOG2N2);
    if (tl == 0) abar[n] = 0;
    const uint32_t bbar = mod_switch(in[n], LOG2N2);
    const uint32_t Lb = (1u + 4u * (__brev((uint32_t)G::template idx<LAST>(tl, 0)) >> (32 - G::LOG))) & (uint32_t)(M - 1);
    __syncthreads();

    double alo[B][E], ahi[B][E];
    {
        const bool direct = kind == JOB_DIRECT;
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int j = G::template idx<0>(tl, m);
            uint64_t v[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int s = (j + h * M + (int)bbar) & (2 * N - 1);
                const uint64_t tv = test_poly<N>(s & (N - 1), direct, lut);
                v[h] = s < N ? tv : (uint64_t)0 - tv;
            }
#pragma unroll
            for (int P = 0; P < B; ++P) {
                alo[P][m] = P == K ? fft::acc_of_torus(v[0]) : 0.0;
                ahi[P][m] = P == K ? fft::acc_of_torus(v[1]) : 0.0;
            }
        }
    }
    constexpr uint32_t GG = (uint32_t)(K + 1) * (K + 1) * M;
    const __amdgpu_buffer_rsrc_t rs = bsk_rsrc(bsk);
    const uint32_t lane_off = 16u * (uint32_t)tl;
    const int steps = (n + 1) / 2;
    FTwr<M, E> twr;
    ftw_load_phase<M, E, 0, FR_TW_SGPR_PAIR>(twr, tw_g, tl);
    // slot m's key values [g][r][c] (Fourier GGSW [r][c][m][lane])
    auto load_keys = [&](double2 (&Bk)[3][2][2], uint32_t sbase, int m) {
#pragma unroll
        for (int gg = 0; gg < 3; ++gg)
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int c = 0; c < 2; ++c)
                    Bk[gg][r][c] =
                        bsk_load(rs, lane_off, sbase + 16u * (gg * GG + (uint32_t)(r * 2 + c) * M + (uint32_t)m * T));
    };
    for (int t = 0; t < steps; ++t) {
        if ((abar[2 * t] | abar[2 * t + 1]) == 0) continue;  // (uniform) X^0 acc - acc = 0
        const uint32_t sbase = (uint32_t)__builtin_amdgcn_readfirstlane(t) * (3u * GG * 16u);
        double2 Bc[3][2][2];
        load_keys(Bc, sbase, 0);  // slot 0 lands during the digits and the forward FFT
        const uint32_t ei = __builtin_amdgcn_readfirstlane((uint32_t)abar[2 * t]);
        const uint32_t ej = __builtin_amdgcn_readfirstlane((uint32_t)abar[2 * t + 1]);
        double2 x[B][E];
#pragma unroll
        for (int P = 0; P < B; ++P)
#pragma unroll
            for (int m = 0; m < E; ++m)
                x[P][m] = make_double2(fft::acc_digit<23>(alo[P][m]), fft::acc_digit<23>(ahi[P][m]));
        fforward_from<M, E, 0, false, true, B, BS>(x, xbuf, twr, nullptr, tl, [](auto) {});
        // slot factors (quadrant table + quarter turns, as the pair shape)
        double bre[2], bim[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t k = __umul24(h == 0 ? ei : ej, Lb) & (2 * N - 1);
            const double2 q = psi[psi_slot((int)(k & (N / 2 - 1)))];
            fft::psi_quadrant(q.x, q.y, k >> (LOG2N2 - 2), bre[h], bim[h]);
        }
#pragma unroll
        for (int m = 0; m < E; ++m) {
            double2 Bn[3][2][2];
            if (m + 1 < E) load_keys(Bn, sbase, m + 1);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t sm = ((m & 1) << 1) | ((m >> 1) & 1);  // brv2(m & 3)
            double cr[3], ci[3];
#pragma unroll
            for (int h = 1; h < 3; ++h) slot_factor(bre[h - 1], bim[h - 1], h == 1 ? ei : ej, sm, cr[h], ci[h]);
            fft::cmul(cr[1], ci[1], cr[2], ci[2], cr[0], ci[0]);
            double2 z[B];
#pragma unroll
            for (int c = 0; c < B; ++c) {  // output column c: K_r = sum_g B_g[r][c] (c_g - 1), own row first
                double kor, koi, kxr, kxi;
#pragma unroll
                for (int gg = 0; gg < 3; ++gg) {
                    const double c1r = cr[gg] - 1.0, c1i = ci[gg];
                    const double2 Bo = Bc[gg][c][c], Bx = Bc[gg][1 - c][c];
                    if (gg == 0) {
                        fft::cmul(Bo.x, Bo.y, c1r, c1i, kor, koi);
                        fft::cmul(Bx.x, Bx.y, c1r, c1i, kxr, kxi);
                    } else {
                        fft::cmac(Bo.x, Bo.y, c1r, c1i, kor, koi);
                        fft::cmac(Bx.x, Bx.y, c1r, c1i, kxr, kxi);
                    }
                }
                double zr, zi;
                fft::cmul(x[c][m].x, x[c][m].y, kor, koi, zr, zi);
                fft::cmac(x[1 - c][m].x, x[1 - c][m].y, kxr, kxi, zr, zi);
                z[c] = make_double2(zr, zi);
            }
#pragma unroll
            for (int c = 0; c < B; ++c) x[c][m] = z[c];
            __builtin_amdgcn_sched_barrier(0);
            if (m + 1 < E) {
#pragma unroll
                for (int gg = 0; gg < 3; ++gg)
#pragma unroll
                    for (int r = 0; r < 2; ++r)
#pragma unroll
                        for (int c = 0; c < 2; ++c) Bc[gg][r][c] = Bn[gg][r][c];
            }
        }
        finverse_from<M, E, LAST, false, true, B, BS>(x, xbuf, twr, nullptr, nullptr, tl);
#pragma unroll
        for (int P = 0; P < B; ++P)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                alo[P][m] = fft::acc_reduce<23>(alo[P][m] + x[P][m].x);
                ahi[P][m] = fft::acc_reduce<23>(ahi[P][m] + x[P][m].y);
            }
    }

    // publish the accumulator as u64 [P][N] over the rows, then sample extract / w-step
    __syncthreads();
    uint64_t* accs = (uint64_t*)xbuf;
    static_assert(8 * B * N <= 16 * B * BS, "dual shape: u64 rows inside the exchange rows");
#pragma unroll
    for (int P = 0; P < B; ++P)
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int j = G::template idx<0>(tl, m);
            accs[P * N + j] = fft::torus_of_acc(alo[P][m]);
            accs[P * N + j + M] = fft::torus_of_acc(ahi[P][m]);
        }
    if (tl < n_out && kind == JOB_MULTI) {
        constexpr int box = N / 16, half = box / 2;
        const uint8_t* lf = lut + 16 * tl;
        uint32_t* terms = wterms + 16 * tl;
        int nt = 0;
        for (int tt = 1; tt <= 16; ++tt) {
            const int d = tt < 16 ? (int)lf[tt] - (int)lf[tt - 1] : -((int)lf[0] + (int)lf[15]);
            if (d != 0) terms[nt++] = (uint32_t)(tt < 16 ? tt * box - half : N - half) | ((uint32_t)(d + 128) << 16);
        }
        wcnt[tl] = nt;
    }
    __syncthreads();
    if (gi >= n_gates) return;
    constexpr int big = K * N;
    if (kind != JOB_MULTI) {
        uint64_t* out = arena + (size_t)gates[gi].out_slot[0] * slot_stride;
        const uint64_t post = kind == JOB_SIGN ? (1ULL << (DELTA_LOG - 1)) : 0;
        for (int c = tl; c <= big; c += NT) {
            const int pp = c < big ? c / N : K, t = c < big ? c % N : 0;
            const int j = t == 0 ? 0 : N - t;
            const uint64_t v = accs[pp * N + j];
            out[c] = (t != 0 ? (uint64_t)0 - v : v) + (c == big ? post : 0);
        }
        return;
    }
    for (int f = 0; f < n_out; ++f) {
        const uint32_t* tf = wterms + 16 * f;
        const int nt = wcnt[f];
        uint64_t* out = arena + (size_t)gates[gi].out_slot[f] * slot_stride;
        for (int c = tl; c <= big; c += NT) {
            const int pp = c < big ? c / N : K, t = c < big ? c % N : 0;
            const int j = t == 0 ? 0 : N - t;
            const uint64_t v = w_step64<N>(accs + pp * N, tf, nt, j);
            out[c] = t != 0 ? (uint64_t)0 - v : v;
        }
    }
}

#ifndef FR_BR_PAIR_TU
// ================================================================== host side
// compiled (k, N) points: the reference's PARAM_MESSAGE_2_CARRY_2 (k = 1, N = 2048) and
// BASELINE's "N = 1024" set (k = 2, N = 1024, the same 2048-bit flattened key)
// k = 1: E = 4 only (its transforms are radix-4 in the inverse, fradix4)
template <int N, int K, int E>
constexpr bool fft_shape_ok() {
#ifdef FR_LAT_E2  // experiment: a 16-wave latency shape (E = 2) for k = 1; host keygen only
    if (K == 1 && N == 2048 && E == 2) return true;
#endif
    return (K == 1 && N == 2048 && E == 4) || (K == 2 && N == 1024 && (E == 4 || E == 8));
}
static bool fft_supported(int K, int N, int E) {
    return (K == 1 && N == 2048 && E == 4) || (K == 2 && N == 1024 && (E == 4 || E == 8));
}

template <int N, int K, int E, bool LAT, int B = 1>
static void fft_attr() {
    static_assert(fbr_smem_bytes<N, K, E, LAT, B>() <= (LAT ? 160 * 1024 : 160 * 1024 / fbr_tp_groups<K, E>()),
                  "LDS per workgroup of the shape");
    FFT_CHECK(hipFuncSetAttribute((const void*)k_blind_rotate_fft<N, K, E, LAT, B>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)fbr_smem_bytes<N, K, E, LAT, B>()));
}

// run body(N, K) with the compile-time ring dimensions of the parameters
template <class F>
static void fft_dispatch(const Params& p, F&& body) {
    if (p.k == 1 && p.N == 2048) body(std::integral_constant<int, 2048>{}, std::integral_constant<int, 1>{});
    else if (p.k == 2 && p.N == 1024) body(std::integral_constant<int, 1024>{}, std::integral_constant<int, 2>{});
    else throw Error(FR_ERR_INVALID, "device: FFT ring needs (k, N) in {(1, 2048), (2, 1024)}");
}

void Device::init_fft() {
    if (p_.k == 2) fft_e_ = 8;  // one wave per polynomial: every transform exchange wave-local
    if (const char* ev = std::getenv("FR_FFT_LANE_ELEMS")) fft_e_ = std::atoi(ev);
    if (const char* ev = std::getenv("FR_FFT_SMALL_BATCH")) fft_small_ = (size_t)std::atol(ev);
    if (const char* ev = std::getenv("FR_FFT_PAIR_BATCH")) fft_pair_ = (size_t)std::atol(ev);
    if (const char* ev = std::getenv("FR_FFT_DUAL")) fft_dual_ = std::atoi(ev) != 0;
    if (p_.k != 1) fft_pair_ = 0;
    if (!fft_supported(p_.k, p_.N, fft_e_))
        throw Error(FR_ERR_INVALID, "device: FFT ring needs (k, N, E) in {(1, 2048, 4), (2, 1024, 4 or 8)}");
    fft_dispatch(p_, [&](auto nc, auto kc) {
        constexpr int N = decltype(nc)::value, K = decltype(kc)::value;
        fft_attr<N, K, 4, true>();
        fft_attr<N, K, 4, false>();
        if constexpr (K == 1) {
            fft_attr<N, K, 4, true, 2>();
            static_assert(fbr_dual_smem_bytes<N>() <= 80 * 1024, "dual shape: two workgroups per CU");
            FFT_CHECK(hipFuncSetAttribute((const void*)k_blind_rotate_fft_dual<N>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)fbr_dual_smem_bytes<N>()));
        }
#ifdef FR_LAT_E2
        if constexpr (fft_shape_ok<N, K, 2>()) fft_attr<N, K, 2, true>();
#endif
        if constexpr (fft_shape_ok<N, K, 8>()) fft_attr<N, K, 8, false>();
    });

    fft::Tables T(p_.N);
    FFT_CHECK(hipMalloc(&d_ftw_, 16 * (size_t)T.M));
    std::vector<fft::c64> psi(2 * (size_t)p_.N);
    for (int k = 0; k < 2 * p_.N; ++k) psi[k] = fft::psi_pow(p_.N, k);
    FFT_CHECK(hipMalloc(&d_fqt_, 16 * psi.size()));
    FFT_CHECK(hipMalloc(&d_fleaf_, 2 * (size_t)T.M));
    FFT_CHECK(hipMemcpy(d_ftw_, T.tw.data(), 16 * (size_t)T.M, hipMemcpyHostToDevice));
    FFT_CHECK(hipMemcpy(d_fqt_, psi.data(), 16 * psi.size(), hipMemcpyHostToDevice));
    FFT_CHECK(hipMemcpy(d_fleaf_, T.leaf.data(), 2 * (size_t)T.M, hipMemcpyHostToDevice));
}

void Device::upload_fft_bsk(const std::vector<uint64_t>& bsk) {
    const int N = p_.N, M = N / 2, kp1 = p_.k + 1;
    const size_t polys = p_.bsk_ggsw() * (size_t)kp1 * kp1;
    fft::Tables tabs(N);
    std::vector<fft::c64> four;
    fft::bsk_to_fourier(tabs, bsk, polys, four);
    // slot order -> per-lane order [poly][m][lane] (one copy per lane geometry E):
    // lane tl's element m is slot idx<LAST>(tl, m), so each load of a wave is 1 KB contiguous
    std::vector<fft::c64> lanes(four.size());
    for (int E : {16, 8, 4, 2}) {
#ifdef FR_LAT_E2
        const bool e2 = E == 2 && p_.k == 1;  // the experiment's latency layout, in the E = 16 slot
#else
        const bool e2 = false;
#endif
        if (E == 2 && !e2) continue;
        double*& dst = d_fbsk_[fbsk_index(E)];
        (void)hipFree(dst);
        dst = nullptr;
        if (!e2 && (!fft_supported(p_.k, N, E) || !fbsk_needed(E))) continue;
        const int T = M / E;
        int e = 0;
        while ((1 << e) < E) ++e;
        const int LAST = (tabs.LOG + e - 1) / e - 1, L = geo_lo(tabs.LOG, e, LAST);
        const int V = fft_layout_variant(tabs.LOG, e);
        std::vector<int> slot((size_t)T * E);
        for (int tl = 0; tl < T; ++tl)
            for (int m = 0; m < E; ++m) slot[(size_t)m * T + tl] = geo_base(tabs.LOG, e, LAST, tl, V) + (m << L);
        for (size_t pq = 0; pq < polys; ++pq)
            for (size_t q = 0; q < (size_t)M; ++q) lanes[pq * M + q] = four[pq * M + slot[q]];
        FFT_CHECK(hipMalloc(&dst, 16 * lanes.size()));
        FFT_CHECK(hipMemcpy(dst, lanes.data(), 16 * lanes.size(), hipMemcpyHostToDevice));
    }
}

void Device::launch_br_fft(const DevGate* d_gates, const uint64_t* d_ks, size_t n, void* stream, void* ev_start,
                           void* ev_stop) {
    const hipStream_t s = (hipStream_t)stream;
    fft_dispatch(p_, [&](auto nc, auto kc) {
        constexpr int N = decltype(nc)::value, K = decltype(kc)::value;
        auto go = [&](auto ec, auto lat, auto bc) {
            constexpr int E = decltype(ec)::value;
            constexpr bool LAT = decltype(lat)::value;
            constexpr int B = decltype(bc)::value;
            if constexpr (fft_shape_ok<N, K, E>() && (B == 1 || K == 1))
                hipExtLaunchKernelGGL(k_blind_rotate_fft<N, K, E, LAT, B>, dim3((unsigned)((n + B - 1) / B)),
                                      dim3(fbr_threads<N, K, E>()), (uint32_t)fbr_smem_bytes<N, K, E, LAT, B>(), s,
                                      (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0, d_ks, p_.ks_stride(), p_.n, d_gates,
                                      (int)n, (const double2*)d_fbsk_[fbsk_index(E)], (const double2*)d_ftw_,
                                      (const double2*)d_fqt_, (const uint16_t*)d_fleaf_, d_arena_, p_.slot_stride());
        };
        using I4 = std::integral_constant<int, 4>;
        using I8 = std::integral_constant<int, 8>;
        using B1 = std::integral_constant<int, 1>;
        // small launches (at most one bootstrap per CU): the latency shape
#ifdef FR_LAT_E2
        if (n <= fft_small_ && K == 1) {
            go(std::integral_constant<int, 2>{}, std::true_type{}, B1{});
            return;
        }
#endif
        if (n <= fft_small_) go(I4{}, std::true_type{}, B1{});
        else if (n <= fft_pair_ && K == 1 && fft_dual_) {
            if constexpr (K == 1)
                hipExtLaunchKernelGGL(k_blind_rotate_fft_dual<N>, dim3((unsigned)n), dim3(N / 8),
                                      (uint32_t)fbr_dual_smem_bytes<N>(), s, (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0,
                                      d_ks, p_.ks_stride(), p_.n, d_gates, (int)n,
                                      (const double2*)d_fbsk_[fbsk_index(4)], (const double2*)d_ftw_,
                                      (const double2*)d_fqt_, (const uint16_t*)d_fleaf_, d_arena_, p_.slot_stride());
        } else if (n <= fft_pair_) go(I4{}, std::true_type{}, std::integral_constant<int, 2>{});  // (k = 1)
        else if (fft_e_ == 4) go(I4{}, std::false_type{}, B1{});
        else go(I8{}, std::false_type{}, B1{});
    });
    FFT_CHECK(hipGetLastError());
}

void Device::free_fft() {
    for (auto& b : d_fbsk_) {
        (void)hipFree(b);
        b = nullptr;
    }
    (void)hipFree(d_ftw_);
    (void)hipFree(d_fqt_);
    (void)hipFree(d_fleaf_);
    d_ftw_ = d_fqt_ = nullptr;
    d_fleaf_ = nullptr;
}

#endif  // !FR_BR_PAIR_TU

}  // namespace fr
