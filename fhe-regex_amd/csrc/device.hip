// HIP kernels for the TFHE gate bootstrap on MI355X (gfx950, CDNA4).
//
//   k_lincomb_keyswitch : lincomb of input LWEs (mod 2^64) fused with the
//                         LWE keyswitch kN -> n (signed base 2^3, 5 levels)
//   k_blind_rotate<N,K,E>: modulus switch, test-polynomial accumulator, n CMUX
//                         steps (rotate -> gadget decompose -> forward NTT ->
//                         MAC with the NTT-domain GGSW -> inverse NTT ->
//                         accumulate), multi-value w-step, sample extract,
//                         Z_Q -> 2^64 conversion.
//   k_bsk_to_ntt<N,K,E> : one-time forward NTT of the bootstrapping key.
//
// Ring: Z_Q[X]/(X^N+1), Q = p0*p1 (rns.h), two 30-bit NTT primes.  One
// workgroup per bootstrap with 2*(K+1)*N/E lanes: each (polynomial, prime)
// pair is owned by N/E lanes (whole waves) holding E residues in registers.
// The log2 N NTT stages run as register-resident phases of log2 E stages
// joined by LDS exchanges.  Butterflies are Harvey-lazy with Montgomery
// products (R = 2^32): forward values stay in [0, 4p), inverse in [0, 2p),
// 32-bit adds and v_min_u32 only.  Twiddles and the BSK are in Montgomery
// form (1/N folded into the BSK); data is in normal form.  The merged-psi
// negacyclic transform: forward Cooley-Tukey with zeta[k] = psi^brv(k),
// outputs in bit-reversed slot order; inverse Gentleman-Sande with
// psi^-brv(k) = -zeta[3*2^s - 1 - k] (negation folded into the butterfly).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <type_traits>

#include "device.h"
#include "geo.h"  // lane geometry and conflict-free LDS maps (shared with fft.hip)
#include "keys.h"
#include "rns.h"

namespace fr {

#define HIP_CHECK(x)                                                                         \
    do {                                                                                     \
        hipError_t _e = (x);                                                                 \
        if (_e != hipSuccess)                                                                \
            throw Error(FR_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(_e) +     \
                                        " at " __FILE__ ":" + std::to_string(__LINE__));     \
    } while (0)

using rns::mont;
using rns::mont_lazy;
using rns::red1;
using rns::red2;

// Montgomery product a*b/2^32 in [0, 2p) (a*b < 4p^2).  (No inline asm in
// this file: the waitcnt pass drains every outstanding load before one.)
__device__ __forceinline__ uint32_t mont_lazy_d(uint32_t a, uint32_t b, uint32_t p, uint32_t pn) {
    return mont_lazy(a, b, p, pn);
}
// Montgomery reduction of a 64-bit sum of products T < 2^63: returns
// T/2^32 mod p as a value below T/2^32 + p (each use states its bound).
__device__ __forceinline__ uint32_t mont_reduce(uint64_t t, uint32_t p, uint32_t pn) {
    const uint32_t m = (uint32_t)t * pn;
    return (uint32_t)((t + (uint64_t)m * p) >> 32);
}

// Harvey-lazy Cooley-Tukey butterfly: x, y in [0, 4p) -> [0, 4p); w Montgomery
// (first = true: x already in [0, 2p), the reduction is skipped)
__device__ __forceinline__ void ct_lazy(uint32_t& x, uint32_t& y, uint32_t w, uint32_t p, uint32_t pn, bool first = false) {
    if (!first) x = red2(x, p);
    const uint32_t t = mont_lazy_d(y, w, p, pn);  // [0, 2p)
    y = x - t + 2 * p;
    x = x + t;
}
// Gentleman-Sande with the flipped twiddle w = -psi^-brv(k):
// (u, v) -> (u + v, (v - u) * w), values in [0, 2p)
__device__ __forceinline__ void gs_lazy(uint32_t& u, uint32_t& v, uint32_t w, uint32_t p, uint32_t pn) {
    const uint32_t s = red2(u + v, p);
    const uint32_t d = v - u + 2 * p;  // (0, 4p)
    v = mont_lazy_d(d, w, p, pn);
    u = s;
}

template <int N, int E, int p>
__device__ __forceinline__ void fwd_phase(uint32_t (&x)[E], const uint32_t* zt, int tl, uint32_t pm, uint32_t pn) {
    using G = NttGeo<N, E>;
    const int b = G::template base<p>(tl);
#pragma unroll
    for (int s = G::s_begin(p); s < G::s_end(p); ++s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
        const uint32_t* zs = zt + (b >> (G::LOG - s));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            ct_lazy(x[m], x[m + dm], zs[(1 << s) + (G::template moff<p>(m) >> (G::LOG - s))], pm, pn, s == 0);
        }
    }
}
template <int N, int E, int p>
__device__ __forceinline__ void inv_phase(uint32_t (&x)[E], const uint32_t* zt, int tl, uint32_t pm, uint32_t pn) {
    using G = NttGeo<N, E>;
    const int b = G::template base<p>(tl);
#pragma unroll
    for (int s = G::s_end(p) - 1; s >= G::s_begin(p); --s) {
        const int dm = 1 << (G::LOG - 1 - s - G::lo(p));
        // zt[3*2^s - 1 - k], k = 2^s + (j >> (LOG-s))
        const uint32_t* zs = zt - (b >> (G::LOG - s));
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (m & dm) continue;
            gs_lazy(x[m], x[m + dm], zs[2 * (1 << s) - 1 - (G::template moff<p>(m) >> (G::LOG - s))], pm, pn);
        }
    }
}
// Does the exchange between phase layouts PF and PT stay inside each wave?
// Lane bit b of phase p holds index bit (b < lo(p) ? b : b + e); the wave
// index is lane bits [6, log2 T).  If those map to the same index bits in both
// layouts, every wave reads back only what it wrote.
template <int N, int E, int PF, int PT>
constexpr bool wave_local() {
    using G = NttGeo<N, E>;
    for (int b = 6; (1 << b) < G::T; ++b) {
        const int f = b < G::lo(PF) ? b : b + G::e, t = b < G::lo(PT) ? b : b + G::e;
        if (f != t) return false;
    }
    return true;
}
// LDS ordering inside one wave: no workgroup barrier, only a compiler fence
// (LDS instructions of a wave execute in order).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// LDS exchange between the layouts of phases PF and PT (row = this lane's
// polynomial).  PRE: a barrier before writing (other waves may still read
// these slots); the barrier after writing is dropped for wave-local exchanges.
template <int N, int E, int PF, int PT, bool PRE = true>
__device__ __forceinline__ void exchange(uint32_t (&x)[E], uint32_t* row, int tl) {
    using G = NttGeo<N, E>;
    constexpr int X = PF < PT ? PF : PT;
    uint32_t* rf = row + G::template at<X>(G::template base<PF>(tl));
    uint32_t* rt = row + G::template at<X>(G::template base<PT>(tl));
    if constexpr (PRE) __syncthreads();
#pragma unroll
    for (int m = 0; m < E; ++m) rf[G::template at<X>(G::template moff<PF>(m))] = x[m];
    if constexpr (wave_local<N, E, PF, PT>() && G::wave_top(PF)) wave_sync();
    else __syncthreads();
#pragma unroll
    for (int m = 0; m < E; ++m) x[m] = rt[G::template at<X>(G::template moff<PT>(m))];
}

// Barrier plan (hazards between waves on the exchange rows).  After any
// exchange every lane reads only slots its own wave owns under the new layout;
// in a wave-top layout those are the wave's own address chunk under every map,
// so a later write of the same layout by the same wave (even under the next
// exchange's map) cannot race another wave.  So only the first exchange of an
// NTT needs a barrier before writing: the forward one follows the rotation
// step (other waves read arbitrary slots of this row), the inverse one follows
// the MAC (other polynomials' waves read this row) -- plus any exchange that
// writes a layout that is not wave-top.
template <int N, int E, int p>
constexpr bool fwd_pre() {
    return p == 0 || !NttGeo<N, E>::wave_top(p);
}
template <int N, int E, int p>
constexpr bool inv_pre() {
    return p == NttGeo<N, E>::NPH - 1 || !NttGeo<N, E>::wave_top(p);
}

template <int N, int E, int X = 0>
constexpr bool exchanges_conflict_free() {
    using G = NttGeo<N, E>;
    if constexpr (X + 1 >= G::NPH) return true;
    else return G::template banks_distinct<X>(X) && G::template banks_distinct<X>(X + 1) &&
                exchanges_conflict_free<N, E, X + 1>();
}

template <int N, int E, int p>
__device__ __forceinline__ void forward_from(uint32_t (&x)[E], uint32_t* row, const uint32_t* zt, int tl, uint32_t pm,
                                             uint32_t pn) {
    fwd_phase<N, E, p>(x, zt, tl, pm, pn);
    if constexpr (p + 1 < NttGeo<N, E>::NPH) {
        exchange<N, E, p, p + 1, fwd_pre<N, E, p>()>(x, row, tl);
        forward_from<N, E, p + 1>(x, row, zt, tl, pm, pn);
    }
}
template <int N, int E, int p>
__device__ __forceinline__ void inverse_from(uint32_t (&x)[E], uint32_t* row, const uint32_t* zt, int tl, uint32_t pm,
                                             uint32_t pn) {
    inv_phase<N, E, p>(x, zt, tl, pm, pn);
    if constexpr (p > 0) {
        exchange<N, E, p, p - 1, inv_pre<N, E, p>()>(x, row, tl);
        inverse_from<N, E, p - 1>(x, row, zt, tl, pm, pn);
    }
}
// natural order (phase-0 layout), values < 2p -> bit-reversed slots (last-phase layout), < 4p
template <int N, int E>
__device__ __forceinline__ void forward_ntt(uint32_t (&x)[E], uint32_t* row, const uint32_t* zt, int tl, uint32_t pm,
                                            uint32_t pn) {
    forward_from<N, E, 0>(x, row, zt, tl, pm, pn);
}
// last-phase layout, values < 2p -> natural order, < 2p; without the 1/N factor
template <int N, int E>
__device__ __forceinline__ void inverse_ntt(uint32_t (&x)[E], uint32_t* row, const uint32_t* zt, int tl, uint32_t pm,
                                            uint32_t pn) {
    inverse_from<N, E, NttGeo<N, E>::NPH - 1>(x, row, zt, tl, pm, pn);
}

// ------------------------------------------------------------ blind rotation
template <int N, int K, int E>
constexpr int br_threads() {
    return 2 * (K + 1) * (N / E);
}
// FR_BR_TIMING (debug builds only, tools/build_variant.sh): wave 0 of workgroup 0
// accumulates s_memtime deltas of the pair-step segments and prints them.
#ifdef FR_BR_TIMING
#define BR_STAMP(k)                                             \
    do {                                                        \
        __builtin_amdgcn_sched_barrier(0);                      \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
        tseg[k] += now_ - tlast;                                \
        tlast = now_;                                           \
        __builtin_amdgcn_sched_barrier(0);                      \
    } while (0)
#else
#define BR_STAMP(k) \
    do {            \
    } while (0)
#endif

// bootstrapping-key unrolling factor (Params::bsk_unroll): pairs for k = 1
template <int K>
constexpr int br_unroll() {
    return K == 1 ? 2 : 1;
}
template <int N, int K, int E>
constexpr size_t br_smem_bytes() {
    return sizeof(uint32_t) * (2 * (size_t)(K + 1) * NttGeo<N, E>::NP + 2 * (size_t)N) + 16 * MAX_OUT + 2 * 1026 +
           4 * 17 * MAX_OUT + (br_unroll<K>() == 2 ? sizeof(uint32_t) * 4 * (size_t)N : 0);
}
constexpr int brv_c(int x, int bits) { return bits == 0 ? 0 : ((x & 1) << (bits - 1)) | brv_c(x >> 1, bits - 1); }
// LDS position of monomial-table entry e (bank swizzle, a permutation within 32-word rows)
__device__ __forceinline__ uint32_t mono_pos(uint32_t e) { return e ^ ((e >> 5) & 31); }

// BSK NTT-domain layout [i][r][c][prime][slot]: natural (bit-reversed) slot
// order, the same for every lane geometry E, so E can be chosen per launch.
template <int N, int E>
__device__ __forceinline__ int bsk_pos(int tl, int m) {
    return NttGeo<N, E>::template idx<NttGeo<N, E>::NPH - 1>(tl, m);
}

// minimum waves per SIMD (register cap 512 / w): 4 -> 128 VGPRs
#ifndef FR_BR_MINW8
#define FR_BR_MINW8 4
#endif
#ifndef FR_BR_MINW16
#define FR_BR_MINW16 4
#endif
template <int E>
constexpr int br_min_waves() {
    return E == 16 ? FR_BR_MINW16 : FR_BR_MINW8;
}

// Multi-value w-step terms of one LUT: w_f = sum_t d_t X^pos_t with
// d = f(m) - f(m-1) at m*box - box/2 and -(f(0) + f(15)) at N - box/2.
// Packed as pos | (d + 128) << 16; returns the count.
template <int N>
__device__ __forceinline__ int lut_terms(const uint8_t* lf, uint32_t* terms) {
    constexpr int box = N / 16, half = box / 2;
    int nt = 0;
    for (int tt = 1; tt <= 16; ++tt) {
        const int d = tt < 16 ? (int)lf[tt] - (int)lf[tt - 1] : -((int)lf[0] + (int)lf[15]);
        if (d != 0) terms[nt++] = (uint32_t)(tt < 16 ? tt * box - half : N - half) | ((uint32_t)(d + 128) << 16);
    }
    return nt;
}
// residue of sum_t d_t (X^pos_t A)[j] mod p from one residue row of A
template <class G>
__device__ __forceinline__ uint32_t w_step(const uint32_t* row, const uint32_t* terms, int nt, int j, uint32_t pm,
                                           int q) {
    constexpr int N = 1 << G::LOG;
    int64_t acc = 0;
    for (int t = 0; t < nt; ++t) {  // nt uniform, terms broadcast from LDS
        const uint32_t tm = terms[t];
        int src = j - (int)(tm & 0xFFFF);
        int d = (int)(tm >> 16) - 128;
        if (src < 0) {
            src += N;
            d = -d;
        }
        acc += (int64_t)d * (int64_t)row[G::template at<0>(src)];
    }
    // |acc| < 16 * 30 * p: shift by 512p before reducing
    return rns::reduce64((uint64_t)(acc + 512LL * pm), q);
}

// Signed gadget digits of the accumulator, split between the two prime lanes
// of each coefficient: the prime-Q lane decomposes elements [Q*E/2, (Q+1)*E/2)
// from both residues, so each digit is computed once.  Round 1 hands the
// sibling the residues it needs, round 2 the digits it did not compute (both in
// this lane's own row, at disjoint slots).  The caller's next write of the row
// (the forward NTT's first exchange) is preceded by a barrier.
#ifndef FR_SPLIT_DIGITS
#define FR_SPLIT_DIGITS 1
#endif
template <int N, int E, int Q>
__device__ __forceinline__ void split_digits(uint32_t (&x)[E], const uint32_t (&acc)[E], uint32_t* row_b0,
                                             const uint32_t* sib_b0, uint32_t pm) {
    using G = NttGeo<N, E>;
    constexpr int HE = E / 2, M0 = Q * HE, O0 = (1 - Q) * HE;
#pragma unroll
    for (int h = 0; h < HE; ++h) row_b0[G::template at<0>(G::template moff<0>(O0 + h))] = acc[O0 + h];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < HE; ++h) {
        const int off = G::template at<0>(G::template moff<0>(M0 + h));
        const uint32_t o = sib_b0[off];
        const int32_t dg = Q ? rns::decompose(o, acc[M0 + h]) : rns::decompose(acc[M0 + h], o);
        row_b0[off] = (uint32_t)dg;
        x[M0 + h] = dg >= 0 ? (uint32_t)dg : (uint32_t)(dg + (int32_t)pm);
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < HE; ++h) {
        const int32_t dg = (int32_t)sib_b0[G::template at<0>(G::template moff<0>(O0 + h))];
        x[O0 + h] = dg >= 0 ? (uint32_t)dg : (uint32_t)(dg + (int32_t)pm);
    }
}

template <int N, int K, int E>
__global__ void __launch_bounds__(2 * (K + 1) * (N / E), br_min_waves<E>())
k_blind_rotate(const uint64_t* __restrict__ ks, int ks_stride, int n, const DevGate* __restrict__ gates,
               const uint32_t* __restrict__ bsk, const uint32_t* __restrict__ tw, uint64_t* __restrict__ arena,
               int slot_stride) {
    using G = NttGeo<N, E>;
    static_assert(exchanges_conflict_free<N, E>(), "LDS maps must make every exchange conflict-free");
    constexpr int NT = br_threads<N, K, E>();
    constexpr int LAST = G::NPH - 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* xbuf = smem;                                // 2(K+1) rows of NP: row (P, q) at (2P + q) * NP
    uint32_t* zt_all = xbuf + 2 * (K + 1) * G::NP;       // 2 x N Montgomery twiddles
    uint8_t* lut = (uint8_t*)(zt_all + 2 * N);           // 16 * n_out
    uint16_t* abar = (uint16_t*)(lut + 16 * MAX_OUT);    // n (<= 1024), zero-padded to even
    uint32_t* wterms = (uint32_t*)(abar + 1026);          // multi-value terms, 16 per output
    int* wcnt = (int*)(wterms + 16 * MAX_OUT);
    uint32_t* mono = (uint32_t*)(wcnt + MAX_OUT);         // unrolled: (psi^e - 1) * R per prime, e < 2N
    constexpr int U = br_unroll<K>();

    const int tid = threadIdx.x;
    const int PQ = __builtin_amdgcn_readfirstlane(tid / G::T), tl = tid % G::T;  // wave-uniform
    const int P = PQ >> 1, q = PQ & 1;
    const uint32_t pm = rns::prime(q), pn = rns::pneg(q);
    const int g = blockIdx.x;
    const uint64_t* in = ks + (size_t)g * ks_stride;

    const int n_out = gates[g].n_out;
    const int kind = gates[g].direct;
    const bool direct = kind == JOB_DIRECT;
    for (int i = tid; i < 2 * N; i += NT) zt_all[i] = tw[i];
    for (int i = tid; i < 16 * n_out; i += NT) lut[i] = gates[g].lut[i / 16][i % 16];
    for (int i = tid; i < n; i += NT) abar[i] = (uint16_t)mod_switch(in[i], G::LOG + 1);
    if (tid == 0) abar[n] = 0;  // pad an odd n
    const uint32_t bbar = mod_switch(in[n], G::LOG + 1);
    if constexpr (U == 2) {
        __syncthreads();  // twiddles loaded
        // X^e in the NTT domain is psi^(e(2 brv(slot) + 1)); psi^e = +-zeta[brv(e mod N)]
        for (int i = tid; i < 4 * N; i += NT) {
            const int qq = i / (2 * N), e = i % (2 * N);
            const uint32_t pq = rns::prime(qq);
            const uint32_t z = zt_all[qq * N + (int)(__brev((uint32_t)(e & (N - 1))) >> (32 - G::LOG))];
            const uint32_t v = e < N ? z : rns::negm(z, pq);
            // (psi^e - 1) * 2^32 mod p, stored XOR-swizzled (mono_pos): within a
            // 32-lane half the lookups are 16 e brv5(l) + c, i.e. two banks; the
            // swizzle spreads them (22.7-way -> 1.95-way average conflict).
            mono[qq * 2 * N + mono_pos(e)] = rns::subm(v, (uint32_t)((1ULL << 32) % pq), pq);
        }
    }
    __syncthreads();
    const uint32_t* zt = zt_all + q * N;

    uint32_t* row = xbuf + PQ * G::NP;
    const uint32_t* row0 = xbuf + (2 * P) * G::NP;  // this polynomial, prime 0
    const uint32_t* row1 = row0 + G::NP;            // ... prime 1
    const int b0 = G::template base<0>(tl), bl = G::template base<LAST>(tl);
    constexpr int XL = G::XL;
    uint32_t* row_b0 = row + G::template at<0>(b0);
    const uint32_t* row0_b0 = row0 + G::template at<0>(b0);
    const uint32_t* row1_b0 = row1 + G::template at<0>(b0);
    uint32_t* row_bl = row + G::template at<XL>(bl);
    const uint32_t* xbuf_q_bl = xbuf + q * G::NP + G::template at<XL>(bl);
    uint32_t acc[E];  // canonical residues, natural order: coefficient idx<0>(tl, m)
    {
        // acc = (0, X^-bbar * V): V's residues into the body rows, then rotate
        constexpr int box = N / 16, half = box / 2;
        if (P == K) {
            const uint32_t dqr = q ? rns::DQR1 : rns::DQR0;
            const uint32_t hq = q ? rns::HQ1 : rns::HQ0;
            for (int jj = tl; jj < N; jj += G::T) {
                uint32_t v = hq;  // multi-value / sign test polynomial (Delta/2) * u
                if (direct) {
                    const int mm = (jj + half) / box;
                    v = mm < 16 ? mont(lut[mm], dqr, pm, pn) : rns::negm(mont(lut[0], dqr, pm, pn), pm);
                }
                row[G::template at<0>(jj)] = v;
            }
        }
        __syncthreads();
        const bool body = P == K;  // mask rows start at zero
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int s = (b0 + G::template moff<0>(m) + (int)bbar) & (2 * N - 1);
            const uint32_t v = row[G::template at<0>(s & (N - 1))];
            acc[m] = body ? (s < N ? v : rns::negm(v, pm)) : 0u;
        }
        __syncthreads();  // the rotated reads above touch slots other waves write next
    }

    const size_t ggsw = (size_t)(K + 1) * (K + 1) * 2 * N;
    if constexpr (U == 1) {
    for (int i = 0; i < n; ++i) {
        const int a = abar[i];
        if (a == 0) continue;  // X^0*acc - acc = 0: exact no-op (uniform branch)
        // 0. prefetch this lane's GGSW_i slots; they land during steps 1-2
        //    (__syncthreads only drains LDS counters, not these loads)
        uint32_t gv[K + 1][E];
        {
            const uint32_t* gi = bsk + (size_t)i * ggsw + (size_t)(P * 2 + q) * N + bl;
#pragma unroll
            for (int r = 0; r <= K; ++r)
#pragma unroll
                for (int m = 0; m < E; ++m) gv[r][m] = gi[(size_t)r * (K + 1) * 2 * N + G::template moff<LAST>(m)];
        }
        // 1. (X^a - 1) * acc, CRT of the two residues, signed gadget digit
        uint32_t x[E];
        // (no barrier before the write: the last inverse exchange left these
        // slots read by this wave only)
#pragma unroll
        for (int m = 0; m < E; ++m) row_b0[G::template at<0>(G::template moff<0>(m))] = acc[m];
        __syncthreads();
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int j = b0 + G::template moff<0>(m);
            const int s = (j - a) & (2 * N - 1);
            const int sp = G::template at<0>(s < N ? s : s - N);
            uint32_t v0 = row0[sp], v1 = row1[sp];
            if (s >= N) {
                v0 = rns::negm(v0, rns::P0);
                v1 = rns::negm(v1, rns::P1);
            }
            const int jo = G::template at<0>(G::template moff<0>(m));
            const int32_t dg = rns::decompose(rns::subm(v0, row0_b0[jo], rns::P0), rns::subm(v1, row1_b0[jo], rns::P1));
            x[m] = dg >= 0 ? (uint32_t)dg : (uint32_t)(dg + (int32_t)pm);
        }
        // 2. forward NTT of this lane group's digit residues
        forward_ntt<N, E>(x, row, zt, tl, pm, pn);
        // 3. external product MAC (in place): x_(P,q) = sum_r D_(r,q) * GGSW_i[r][P][q]
        //    (no barrier before the write: these slots were last read by this wave)
#pragma unroll
        for (int m = 0; m < E; ++m) row_bl[G::template at<XL>(G::template moff<LAST>(m))] = x[m];
        __syncthreads();
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int po = G::template at<XL>(G::template moff<LAST>(m));
            // sum_r D_r B_r in 64 bits (< 3 * 4p * p = 12p^2, and p < 0.235 * 2^32):
            // one reduction to [0, 3.9p), one conditional subtraction to [0, 2p)
            uint64_t ss = 0;
#pragma unroll
            for (int r = 0; r <= K; ++r) {
                const uint32_t d = (r == P) ? x[m] : xbuf_q_bl[2 * r * G::NP + po];
                ss += (uint64_t)d * gv[r][m];
            }
            x[m] = red2(mont_reduce(ss, pm, pn), pm);
        }
        // 4. inverse NTT and accumulate (1/N is folded into the BSK)
        inverse_ntt<N, E>(x, row, zt, tl, pm, pn);
#pragma unroll
        for (int m = 0; m < E; ++m) acc[m] = red1(red1(x[m], pm) + acc[m], pm);
    }
    } else {
    // Unrolled blind rotation: one step per pair (i, j) = (2t, 2t+1),
    //   acc += sum_g (X^e_g - 1) * (GGSW_3t+g [x] acc),  e = (a_i + a_j, a_i, a_j),
    // with one decomposition of acc, one forward NTT per polynomial, the three
    // monomial factors applied slot-wise in the NTT domain, one inverse NTT.
    const uint32_t* sib_b0 = xbuf + (2 * P + (1 - q)) * G::NP + G::template at<0>(b0);  // other prime, same polynomial
    const uint32_t* mono_q = mono + q * 2 * N;
    const uint32_t B0 = 2 * (__brev((uint32_t)bl) >> (32 - G::LOG)) + 1;  // slot bl + moff: 2 brv + 1 = B0 + c_m
    const int steps = (n + 1) / 2;
#ifdef FR_BR_TIMING
    uint64_t tseg[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t tlast = __builtin_amdgcn_s_memtime();
    const uint64_t tstart = tlast;
#endif
    for (int t = 0; t < steps; ++t) {
        const uint32_t ai = abar[2 * t], aj = abar[2 * t + 1];
        if ((ai | aj) == 0) continue;  // X^0*acc - acc = 0 (uniform branch)
        BR_STAMP(0);
        // 0. prefetch the three GGSWs of this pair
        uint32_t gv[3][K + 1][E];
        {
            const uint32_t* gi = bsk + (size_t)(3 * t) * ggsw + (size_t)(P * 2 + q) * N + bl;
#pragma unroll
            for (int gg = 0; gg < 3; ++gg)
#pragma unroll
                for (int r = 0; r <= K; ++r)
#pragma unroll
                    for (int m = 0; m < E; ++m)
#ifdef FR_BR_NOBSK  // timing experiment only: no GGSW traffic (wrong results)
                        gv[gg][r][m] = (uint32_t)(t + gg + r + m);
#else
                        gv[gg][r][m] = gi[(size_t)gg * ggsw + (size_t)r * (K + 1) * 2 * N + G::template moff<LAST>(m)];
#endif
        }
        // 1. signed gadget digits of acc, split between the two prime lanes of a
        //    coefficient (residues and digits swapped through LDS)
        uint32_t x[E];
#if FR_SPLIT_DIGITS
        if (q == 0) split_digits<N, E, 0>(x, acc, row_b0, sib_b0, pm);
        else split_digits<N, E, 1>(x, acc, row_b0, sib_b0, pm);
#else
#pragma unroll
        for (int m = 0; m < E; ++m) row_b0[G::template at<0>(G::template moff<0>(m))] = acc[m];
        __syncthreads();
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const uint32_t o = sib_b0[G::template at<0>(G::template moff<0>(m))];
            const int32_t dg = q ? rns::decompose(o, acc[m]) : rns::decompose(acc[m], o);
            x[m] = dg >= 0 ? (uint32_t)dg : (uint32_t)(dg + (int32_t)pm);
        }
#endif
        BR_STAMP(1);
        // 2. forward NTT (its first exchange waits for the sibling reads above)
        forward_ntt<N, E>(x, row, zt, tl, pm, pn);
        BR_STAMP(2);
        // 3. MAC with the three GGSWs and their monomial factors
#pragma unroll
        for (int m = 0; m < E; ++m) row_bl[G::template at<XL>(G::template moff<LAST>(m))] = x[m];
        __syncthreads();
        BR_STAMP(6);
        const uint32_t e[3] = {(ai + aj) & (2 * N - 1), ai, aj};
        uint32_t eb[3];
#pragma unroll
        for (int gg = 0; gg < 3; ++gg) eb[gg] = __builtin_amdgcn_readfirstlane(e[gg]) * B0;
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int po = G::template at<XL>(G::template moff<LAST>(m));
            uint32_t d[K + 1];
#pragma unroll
            for (int r = 0; r <= K; ++r) d[r] = (r == P) ? x[m] : xbuf_q_bl[2 * r * G::NP + po];
            // y_g = sum_r D_r B_gr as one 64-bit sum (d < 4p, B < p: < 8p^2; with
            // p < 0.235 * 2^32 one reduction lands in [0, 2.87p)); then
            // z = sum_g y_g (psi^e_g - 1) < 8.6p^2 < 2^63, one reduction to
            // [0, 3p) and one subtraction of 2p: [0, 2p).
            uint64_t zs = 0;
#pragma unroll
            for (int gg = 0; gg < 3; ++gg) {
                uint64_t ys = 0;
#pragma unroll
                for (int r = 0; r <= K; ++r) ys += (uint64_t)d[r] * gv[gg][r][m];
                const uint32_t y = mont_reduce(ys, pm, pn);  // [0, 2.87p)
                const uint32_t ex = (eb[gg] + e[gg] * (uint32_t)(2 * brv_c(G::template moff<LAST>(m), G::LOG))) & (2 * N - 1);
                zs += (uint64_t)y * mono_q[mono_pos(ex)];
            }
            x[m] = red1(mont_reduce(zs, pm, pn), 2 * pm);  // [0, 3p) -> [0, 2p)
        }
        BR_STAMP(3);
        // 4. inverse NTT and accumulate (1/N is folded into the BSK)
        inverse_ntt<N, E>(x, row, zt, tl, pm, pn);
        BR_STAMP(4);
#pragma unroll
        for (int m = 0; m < E; ++m) acc[m] = red1(red1(x[m], pm) + acc[m], pm);
        BR_STAMP(5);
    }
#ifdef FR_BR_TIMING
    if (blockIdx.x == 0 && tid == 0)
        printf("BR_TIMING E=%d steps=%d total=%lu decomp=%lu fwd=%lu mac_wait=%lu mac=%lu inv=%lu acc=%lu top=%lu\n", E,
               steps, (unsigned long)(__builtin_amdgcn_s_memtime() - tstart), (unsigned long)tseg[1],
               (unsigned long)tseg[2], (unsigned long)tseg[6], (unsigned long)tseg[3], (unsigned long)tseg[4],
               (unsigned long)tseg[5], (unsigned long)tseg[0]);
#endif
    }

    // publish the accumulator: the outputs need both residues of a coefficient
    __syncthreads();
#pragma unroll
    for (int m = 0; m < E; ++m) row_b0[G::template at<0>(G::template moff<0>(m))] = acc[m];
    __syncthreads();
    const int big = K * N;
    if (kind != JOB_MULTI) {
        // sample extract (coefficient 0) under the flattened key, then Z_Q -> 2^64
        uint64_t* out = arena + (size_t)gates[g].out_slot[0] * slot_stride;
        // sign gate: +-Delta/2 (+ Delta/2) -> {0, Delta}
        const uint64_t post = kind == JOB_SIGN ? (1ULL << (DELTA_LOG - 1)) : 0;
        for (int c = tid; c <= big; c += NT) {
            const int pp = c < big ? c / N : K, t = c < big ? c % N : 0;
            const int j = t == 0 ? 0 : N - t;
            const uint32_t* r0 = xbuf + 2 * pp * G::NP;
            const int aj = G::template at<0>(j);
            uint32_t v0 = r0[aj], v1 = r0[G::NP + aj];
            if (t != 0) {
                v0 = rns::negm(v0, rns::P0);
                v1 = rns::negm(v1, rns::P1);
            }
            out[c] = rns::to_torus(v0, v1) + (c == big ? post : 0);
        }
        return;
    }
    // multi-value: acc_f = w_f * acc with w_f = sum_t d_t X^{pos_t} (small d_t)
    if (tid < n_out) wcnt[tid] = lut_terms<N>(lut + 16 * tid, wterms + 16 * tid);
    __syncthreads();
    for (int f = 0; f < n_out; ++f) {
        const uint32_t* tf = wterms + 16 * f;
        const int nt = wcnt[f];
        uint64_t* out = arena + (size_t)gates[g].out_slot[f] * slot_stride;
        for (int c = tid; c <= big; c += NT) {
            const int pp = c < big ? c / N : K, t = c < big ? c % N : 0;
            const int j = t == 0 ? 0 : N - t;
            const uint32_t* r0 = xbuf + 2 * pp * G::NP;
            uint32_t v0 = w_step<G>(r0, tf, nt, j, rns::P0, 0), v1 = w_step<G>(r0 + G::NP, tf, nt, j, rns::P1, 1);
            if (t != 0) {
                v0 = rns::negm(v0, rns::P0);
                v1 = rns::negm(v1, rns::P1);
            }
            out[c] = rns::to_torus(v0, v1);
        }
    }
}

// ------------------------------------------------------ BSK -> NTT domain
// block = (i, r); lanes (c, prime): residue of the mod-Q coefficient, to
// Montgomery form, forward NTT, canonical, times 1/N.
template <int N, int K, int E>
__global__ void __launch_bounds__(2 * (K + 1) * (N / E))
k_bsk_to_ntt(const uint64_t* __restrict__ coef, const uint32_t* __restrict__ tw, uint32_t ninv_r0, uint32_t ninv_r1,
             uint32_t* __restrict__ out) {
    using G = NttGeo<N, E>;
    constexpr int NT = br_threads<N, K, E>();
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* xbuf = smem;
    uint32_t* zt_all = xbuf + 2 * (K + 1) * G::NP;
    const int tid = threadIdx.x, PQ = __builtin_amdgcn_readfirstlane(tid / G::T), tl = tid % G::T;
    const int P = PQ >> 1, q = PQ & 1;
    const uint32_t pm = rns::prime(q), pn = rns::pneg(q);
    const uint32_t r2 = q ? rns::R2_1 : rns::R2_0, ninv = q ? ninv_r1 : ninv_r0;
    for (int i = tid; i < 2 * N; i += NT) zt_all[i] = tw[i];
    __syncthreads();
    const size_t poly = (size_t)blockIdx.x * (K + 1) + P;  // blockIdx.x = i*(K+1) + r
    uint32_t x[E];
#pragma unroll
    for (int m = 0; m < E; ++m) x[m] = mont(rns::reduce64(coef[poly * N + G::template idx<0>(tl, m)], q), r2, pm, pn);
    forward_ntt<N, E>(x, xbuf + PQ * G::NP, zt_all + q * N, tl, pm, pn);
#pragma unroll
    for (int m = 0; m < E; ++m) out[(poly * 2 + q) * N + bsk_pos<N, E>(tl, m)] = mont(red1(red2(x[m], pm), pm), ninv, pm, pn);
}

// ------------------------------------------------ ring product (parity test)
// lanes (operand, prime); product of a, b in [0, Q) mod Q
template <int N, int E>
__global__ void __launch_bounds__(4 * (N / E))
k_ring_mul(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, const uint32_t* __restrict__ tw,
           uint32_t r2n0, uint32_t r2n1, uint64_t* __restrict__ out) {
    using G = NttGeo<N, E>;
    constexpr int LAST = G::NPH - 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* xbuf = smem;  // rows (operand, prime)
    uint32_t* zt_all = xbuf + 4 * G::NP;
    const int tid = threadIdx.x, PQ = __builtin_amdgcn_readfirstlane(tid / G::T), tl = tid % G::T;
    const int P = PQ >> 1, q = PQ & 1;
    const uint32_t pm = rns::prime(q), pn = rns::pneg(q);
    for (int i = tid; i < 2 * N; i += 4 * G::T) zt_all[i] = tw[i];
    __syncthreads();
    const uint32_t* zt = zt_all + q * N;
    const uint64_t* src = (P == 0 ? a : b) + (size_t)blockIdx.x * N;
    uint32_t x[E];
#pragma unroll
    for (int m = 0; m < E; ++m) x[m] = rns::reduce64(src[G::template idx<0>(tl, m)], q);
    uint32_t* row = xbuf + PQ * G::NP;
    forward_ntt<N, E>(x, row, zt, tl, pm, pn);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < E; ++m) row[G::template at<G::XL>(G::template idx<LAST>(tl, m))] = x[m];
    __syncthreads();
    // a*b/R, then * R^2/N / R
    const uint32_t r2n = q ? r2n1 : r2n0;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int pos = G::template at<G::XL>(G::template idx<LAST>(tl, m));
        const uint32_t u = red1(red2(xbuf[q * G::NP + pos], pm), pm);  // operand a, canonical
        x[m] = mont(mont_lazy(u, xbuf[(2 + q) * G::NP + pos], pm, pn), r2n, pm, pn);
    }
    inverse_ntt<N, E>(x, row, zt, tl, pm, pn);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < E; ++m) row[G::template at<0>(G::template idx<0>(tl, m))] = red1(x[m], pm);
    __syncthreads();
    for (int c = tid; c < N; c += 4 * G::T)
        out[(size_t)blockIdx.x * N + c] = rns::crt(xbuf[G::template at<0>(c)], xbuf[G::NP + G::template at<0>(c)]);
}

// ------------------------------------------------- lincomb + keyswitch
// Tile: 32 gates x 64 output columns x one slice of the kN input coefficients
// per 256-thread workgroup (split-K: the slices' partial sums are exact mod
// 2^64, so they are combined with 64-bit atomic adds into a zeroed output).
// Each wave owns 8 gates; each lane one output column.  Digits of the
// lincomb'd mask coefficients are staged in LDS per chunk of 32 coefficients;
// KSK rows are read once per tile, coalesced (64 consecutive u64 per wave).
constexpr int KS_BT = 32, KS_CT = 64, KS_CH = 32;

// arena slot of a gate input: s >= 0 is a slot; s < 0 a content reference of a
// template plan, resolved through the bound content map (Device::bind_content)
__device__ __forceinline__ int arena_slot(int s, const int* __restrict__ cmap) { return s >= 0 ? s : cmap[-1 - s]; }

template <int KSB, int KSL>
__global__ void __launch_bounds__(256)
k_lincomb_keyswitch(const DevGate* __restrict__ gates, int B, const uint64_t* __restrict__ arena, int slot_stride,
                    const int* __restrict__ cmap, const uint64_t* __restrict__ ksk, int n, int big,
                    int chunks_per_split, unsigned long long* __restrict__ out, int out_stride) {
    __shared__ int8_t dig[KS_BT][KS_CH][KSL];
    __shared__ DevGate sg[KS_BT];
    const int tid = threadIdx.x;
    const int col = blockIdx.y * KS_CT + (tid & 63);
    const int rg = tid >> 6;
    const int b0 = blockIdx.x * KS_BT;
    const int c_begin = blockIdx.z * chunks_per_split * KS_CH;
    const int c_end = min(big, c_begin + chunks_per_split * KS_CH);
    for (int e = tid; e < KS_BT; e += 256) {
        if (b0 + e < B) {
            sg[e] = gates[b0 + e];
            for (int q = 0; q < sg[e].n_in; ++q) sg[e].in_slot[q] = arena_slot(sg[e].in_slot[q], cmap);
        } else {
            sg[e].n_in = 0, sg[e].offset = 0;
        }
    }
    uint64_t acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = 0;
    for (int i0 = c_begin; i0 < c_end; i0 += KS_CH) {
        __syncthreads();
        for (int e = tid; e < KS_BT * KS_CH; e += 256) {
            const int row = e / KS_CH, ii = e % KS_CH;
            uint64_t v = 0;
            if (i0 + ii < c_end) {
                const DevGate& gg = sg[row];
                for (int q = 0; q < gg.n_in; ++q)
                    v += (uint64_t)(int64_t)gg.in_w[q] * arena[(size_t)gg.in_slot[q] * slot_stride + i0 + ii];
            }
            int32_t d[KSL];
            ks_decompose<KSB, KSL>(v, d);
#pragma unroll
            for (int j = 0; j < KSL; ++j) dig[row][ii][j] = (int8_t)d[j];
        }
        __syncthreads();
        if (col <= n) {
            const int lim = c_end - i0 < KS_CH ? c_end - i0 : KS_CH;
            for (int ii = 0; ii < lim; ++ii) {
#pragma unroll
                for (int j = 0; j < KSL; ++j) {
                    const uint64_t kv = ksk[((size_t)(i0 + ii) * KSL + j) * (n + 1) + col];
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const int64_t d = dig[rg * 8 + r][ii][j];
                        acc[r] -= (uint64_t)d * kv;
                    }
                }
            }
        }
    }
    if (col <= n) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int row = rg * 8 + r, b = b0 + row;
            if (b >= B) continue;
            uint64_t v = acc[r];
            if (col == n && blockIdx.z == 0) {
                const DevGate& gg = sg[row];
                uint64_t body = (uint64_t)(int64_t)gg.offset << (DELTA_LOG - 1);
                for (int q = 0; q < gg.n_in; ++q)
                    body += (uint64_t)(int64_t)gg.in_w[q] * arena[(size_t)gg.in_slot[q] * slot_stride + big];
                v += body;
            }
            if (gridDim.z == 1) out[(size_t)b * out_stride + col] = v;
            else atomicAdd(&out[(size_t)b * out_stride + col], (unsigned long long)v);
        }
    }
}

// ------------------------------------------- keyswitch on int8 MFMA
// out[g][t] = [t == n] * body_g - sum_k D[g][k] * KSK[k][t]  (mod 2^64), with
// D the signed base-2^3 digits of the lincomb'd mask (|d| <= 4, k = 5i + level)
// and KSK split into 8 balanced byte limbs, KSK = sum_l L_l * 256^l (mod 2^64),
// L_l in [-128, 128).  Each sum_k D * L_l is an exact i32 GEMM (|.| <= 4 * 128 *
// 10240 < 2^31) on v_mfma_i32_32x32x32_i8; limbs recombine in the epilogue.
// Layouts: D (Bp rows: B rounded up to the wave's row tiles, zero rows) and L (limb
// column col*8 + l, padded with zero columns) in MFMA fragment order: the operand of
// (32-row tile, 32-k tile) is 1 KB contiguous, lane r + 32h holding row r, k = 16h..16h+15,
// so every fragment load of a wave is one fully coalesced 1 KB read.
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));
// byte offset of (row, k) in a fragment-ordered operand with KT = KD / 32 k tiles
__device__ __forceinline__ size_t ks_frag(int row, int k, int KT) {
    return ((((size_t)(row >> 5) * KT + (k >> 5)) * 64 + (row & 31) + 32 * ((k >> 4) & 1)) << 4) + (k & 15);
}

// lincomb + digits: one thread per (gate, input coefficient); the body per gate.
// The same launch zeroes the mask words of each output row (the MFMA pass
// subtracts into them with atomics) and the padding digit rows B <= g < gridDim.y.
template <int KSB, int KSL>
__global__ void __launch_bounds__(256)
k_ks_digits(const DevGate* __restrict__ gates, int B, const uint64_t* __restrict__ arena, int slot_stride,
            const int* __restrict__ cmap, int big, int8_t* __restrict__ dig, uint64_t* __restrict__ ks, int ks_n,
            int ks_stride) {
    const int g = blockIdx.y, KT = big * KSL / 32;
    if (g >= B) {  // padding row of the last row tile: zero digits (16-byte halves of its fragments)
        for (int i = blockIdx.x * 256 + threadIdx.x; i < 2 * KT; i += gridDim.x * 256)
            *(int4*)(dig + ks_frag(g, 16 * i, KT)) = int4{0, 0, 0, 0};
        return;
    }
    const DevGate& gg = gates[g];
    const int nin = gg.n_in;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < ks_n; t += gridDim.x * 256) ks[(size_t)g * ks_stride + t] = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i <= big; i += gridDim.x * 256) {
        uint64_t v = i == big ? (uint64_t)(int64_t)gg.offset << (DELTA_LOG - 1) : 0;
        for (int q = 0; q < nin; ++q)
            v += (uint64_t)(int64_t)gg.in_w[q] * arena[(size_t)arena_slot(gg.in_slot[q], cmap) * slot_stride + i];
        if (i == big) {
            ks[(size_t)g * ks_stride + ks_n] = v;  // column n of the output row; the MFMA pass subtracts
        } else {
            int32_t d[KSL];
            ks_decompose<KSB, KSL>(v, d);
#pragma unroll
            for (int j = 0; j < KSL; ++j) dig[ks_frag(g, i * KSL + j, KT)] = (int8_t)d[j];
        }
    }
}

// The same pass, one workgroup per gate and sixteen consecutive coefficients per thread: its
// 16 KSL digits are KSL whole 16-byte pieces of the fragment-ordered digit row (k = 16 KSL q ..
// 16 KSL q + 16 KSL - 1 starts a piece), stored as 16-byte writes, where k_ks_digits's byte
// stores scatter every digit over 16-byte pieces of 10 fragments; the inputs load as 16-byte
// vectors.  (needs big % 16 == 0)  The inputs' slot lookups (content map included) and their
// body coefficients are fetched by one thread per input at once, and the mask loads of four
// inputs are in flight together: with one input at a time, a small level's fan-in-16 gates
// paid sixteen dependent memory round trips (≈19 µs per launch at 1-16 gates).
template <int KSB, int KSL>
__global__ void __launch_bounds__(128)
k_ks_digits16(const DevGate* __restrict__ gates, int B, const uint64_t* __restrict__ arena, int slot_stride,
              const int* __restrict__ cmap, int big, int8_t* __restrict__ dig, uint64_t* __restrict__ ks, int ks_n,
              int ks_stride) {
    const int g = blockIdx.x, KT = big * KSL / 32, groups = big / 16;
    if (g >= B) {  // padding row of the last row tile: zero digits
        for (int q = threadIdx.x; q < groups; q += blockDim.x)
#pragma unroll
            for (int c = 0; c < KSL; ++c) *(int4*)(dig + ks_frag(g, 16 * (q * KSL + c), KT)) = int4{0, 0, 0, 0};
        return;
    }
    __shared__ int slot_s[16];
    __shared__ uint64_t w_s[16], body_s[16];
    const DevGate& gg = gates[g];
    const int nin = gg.n_in;
    if (threadIdx.x < nin) {
        const int i = threadIdx.x;
        const int slot = arena_slot(gg.in_slot[i], cmap);
        const uint64_t w = (uint64_t)(int64_t)gg.in_w[i];
        slot_s[i] = slot;
        w_s[i] = w;
        body_s[i] = w * arena[(size_t)slot * slot_stride + big];
    }
    for (int t = threadIdx.x; t < ks_n; t += blockDim.x) ks[(size_t)g * ks_stride + t] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {  // column n of the output row (the body); the MFMA pass subtracts
        uint64_t v = (uint64_t)(int64_t)gg.offset << (DELTA_LOG - 1);
        for (int q = 0; q < nin; ++q) v += body_s[q];
        ks[(size_t)g * ks_stride + ks_n] = v;
    }
    for (int q = threadIdx.x; q < groups; q += blockDim.x) {
        uint64_t v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = 0;
        int qi = 0;
        for (; qi + 4 <= nin; qi += 4) {  // four inputs' loads in flight
            ulonglong2 x[4][8];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const ulonglong2* src = (const ulonglong2*)(arena + (size_t)slot_s[qi + u] * slot_stride + 16 * q);
#pragma unroll
                for (int e = 0; e < 8; ++e) x[u][e] = src[e];
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the 32 loads ahead of their first use
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t w = w_s[qi + u];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[2 * e] += w * x[u][e].x;
                    v[2 * e + 1] += w * x[u][e].y;
                }
            }
        }
        for (; qi < nin; ++qi) {
            const uint64_t w = w_s[qi];
            const ulonglong2* src = (const ulonglong2*)(arena + (size_t)slot_s[qi] * slot_stride + 16 * q);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const ulonglong2 x = src[e];
                v[2 * e] += w * x.x;
                v[2 * e + 1] += w * x.y;
            }
        }
        uint32_t words[4 * KSL];
#pragma unroll
        for (int b = 0; b < 4 * KSL; ++b) words[b] = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            int32_t d[KSL];
            ks_decompose<KSB, KSL>(v[e], d);
#pragma unroll
            for (int j = 0; j < KSL; ++j) {
                const int byte = e * KSL + j;
                words[byte >> 2] |= (uint32_t)(uint8_t)(int8_t)d[j] << (8 * (byte & 3));
            }
        }
#pragma unroll
        for (int c = 0; c < KSL; ++c)
            *(uint4*)(dig + ks_frag(g, 16 * (q * KSL + c), KT)) =
                uint4{words[4 * c], words[4 * c + 1], words[4 * c + 2], words[4 * c + 3]};
    }
}

// one wave per MR x 1 tiles of 32 x 32 (gate, limb-column) and one K slice
// (z of GZ); 4 waves per workgroup along the column direction
// share the gate rows through L1, and the MR row tiles of a wave share each KSK
// fragment (MR-fold less KSK traffic).  Partial results are subtracted from out
// (pre-set to [t == n] * body) with 64-bit atomics: exact mod 2^64 in any order.
// Workgroup order (one-dimensional grid, XCD-aware).  The hardware deals workgroup b to
// XCD b % 8; XCD j takes the column groups [j GYX, (j+1) GYX) for every row group and
// K slice, so each KSK limb fragment is fetched into one XCD's L2 only, and the row
// groups of that XCD (dispatched next to each other: row group fastest) read it there.
// Without the remap, the row groups of a column group sat on different XCDs and each
// fetched the whole limb matrix (4x the KSK traffic at 512 gates).  xcd == 0: the plain
// order (row group fastest, then column group, then K slice) for A/B runs.
struct KsTile {
    int x, y, z;
};
__device__ __forceinline__ bool ks_tile(int b, int GX, int GY, int GZ, int xcd, KsTile& t) {
    if (!xcd) {
        t.x = b % GX, t.y = (b / GX) % GY, t.z = b / (GX * GY);
        return t.z < GZ;
    }
    const int GYX = (GY + 7) / 8, loc = b >> 3;
    t.x = loc % GX;
    t.z = (loc / GX) % GZ;
    t.y = (b & 7) * GYX + loc / (GX * GZ);
    return loc < GX * GZ * GYX && t.y < GY;
}
__host__ __device__ inline int ks_grid_blocks(int GX, int GY, int GZ, int xcd) {
    return xcd ? 8 * GX * GZ * ((GY + 7) / 8) : GX * GY * GZ;
}

// k-steps per stage of the LDS-DMA ring of k_ks_glds
#ifndef FR_KS_SK
#define FR_KS_SK 2
#endif
// stages in the LDS-DMA ring of k_ks_glds (NB - 1 in flight)
#ifndef FR_KS_NB
#define FR_KS_NB 4
#endif
// (k_ks_mfma: k-steps in flight per wave, 8 with one row tile, 2 with four; four with four
// row tiles took 512 gates from 100 to 158 us of keyswitch: the registers cost occupancy)
// limb l of KSK column t sits at limb column 8 t + l (the MFMA's column operand), so the 8
// limbs of a column land in 8 adjacent lanes of the accumulator.  (Measured and dropped in
// round 3: the limbs as the row operand, each lane recombining two whole columns in
// registers -- its atomics then scatter over 32 gate rows per instruction, 4x the memory-side
// atomic transactions: 512 gates 73 -> 83 us.)
__host__ __device__ inline int ks_limb_col(int t, int l) { return t * 8 + l; }
// one MFMA step of a wave: acc += (32 digit rows) x (32 limb columns), k = 32
__device__ __forceinline__ v16i_t ks_mma(v4i_t a, v4i_t b, v16i_t acc) {
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
}
// a 64-bit value from another lane of the row by a DPP move (dpp_ctrl CTRL, all rows and banks)
template <int CTRL>
__device__ __forceinline__ uint64_t ks_dpp64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ bool lane_is_zero(int r, int h) { return r == 0 && h == 0; }
// Epilogue: recombine the 8 byte limbs of each KSK column and subtract the wave's MR x MC
// tiles from out (pre-set to [t == n] * body) with 64-bit atomics (exact mod 2^64 in any
// order, so K slices meet there).  Rows g0 + 32 t, limb columns lcw + 32 c.
template <int MR, int MC>
__device__ __forceinline__ void ks_epilogue(const v16i_t (&acc)[MR][MC], int g0, int lcw, int r, int h, int B, int ncols,
                                            int nlc, unsigned long long* __restrict__ out, int out_stride) {
    // lane holds D[row][lc + r] for rows (i&3) + 8(i>>2) + 4h: limb l = r & 7 of
    // column (lc + r) / 8; the 8 limbs of a column meet across the lane's 8-lane group
    const int limb = r & 7;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int lc = lcw + 32 * c, col = (lc + r) >> 3;
        if (lc >= nlc) continue;  // uniform
#pragma unroll
        for (int t = 0; t < MR; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                uint64_t v = (uint64_t)(int64_t)acc[t][c][i] << (8 * limb);
                // sum over the 8 lanes of the column: DPP lane moves (quad_perm [1,0,3,2],
                // [2,3,0,1], then row_half_mirror pairs the two quads of each 8-lane group)
                v += ks_dpp64<0xB1>(v);
                v += ks_dpp64<0x4E>(v);
                v += ks_dpp64<0x141>(v);
                const int g = g0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
#if defined(FR_KS_TIMING_STORE)  // timing experiment only (wrong results with K slices): plain stores
                if (limb == 0 && g < B && col < ncols) out[(size_t)g * out_stride + col] = 0 - v;
#elif defined(FR_KS_TIMING_NOEPI)  // timing experiment only: one store per wave instead of the epilogue
                if (i == 0 && t == 0 && c == 0 && lane_is_zero(r, h)) out[(size_t)g0 * out_stride] = v;
                continue;
#else
                if (limb == 0 && g < B && col < ncols && v != 0)
                    atomicAdd(&out[(size_t)g * out_stride + col], (unsigned long long)(0 - v));
#endif
            }
    }
}

template <int MR, int MC>
__global__ void __launch_bounds__(256)
k_ks_mfma(const int8_t* __restrict__ dig, const int8_t* __restrict__ kl, int B, int KD, int ncols /* n + 1 */,
          int nlc /* limb-columns, multiple of 32 */, unsigned long long* __restrict__ out, int out_stride, int GX,
          int GY, int GZ, int xcd) {
    constexpr int UN = MR * MC == 1 ? 8 : 2;  // k-steps in flight per wave
    KsTile tile;
    if (!ks_tile((int)blockIdx.x, GX, GY, GZ, xcd, tile)) return;  // padding workgroup (uniform)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int g0 = tile.x * 32 * MR;
    const int lcw = (tile.y * 4 + w) * 32 * MC;  // first limb-column of this wave's MC column tiles
    if (lcw >= nlc) return;  // whole wave
    const int kspan = KD / GZ, kb = tile.z * kspan, KT = KD / 32;
    // fragment (tile, k) at ((tile * KT + k / 32) * 64 + lane) * 16: one k step of 32 is 1 KB
    const int8_t* ap = dig + ((size_t)(g0 >> 5) * KT * 64 + lane) * 16 + (size_t)kb * 32;
    const int8_t* bp[MC];
#pragma unroll
    for (int c = 0; c < MC; ++c)  // a tile past the padded columns re-reads the last one (its result is dropped)
        bp[c] = kl + ((size_t)(min(lcw + 32 * c, nlc - 32) >> 5) * KT * 64 + lane) * 16 + (size_t)kb * 32;
    v16i_t acc[MR][MC];
#pragma unroll
    for (int t = 0; t < MR; ++t)
#pragma unroll
        for (int c = 0; c < MC; ++c) acc[t][c] = v16i_t{0};
    for (int k0 = 0; k0 < kspan; k0 += 32 * UN) {  // kspan is a multiple of 256 (host)
        v4i_t a[UN][MR], b[UN][MC];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
#pragma unroll
            for (int c = 0; c < MC; ++c) b[u][c] = *(const v4i_t*)(bp[c] + (size_t)(k0 + 32 * u) * 32);
#pragma unroll
            for (int t = 0; t < MR; ++t) a[u][t] = *(const v4i_t*)(ap + (size_t)t * KD * 32 + (size_t)(k0 + 32 * u) * 32);
        }
#pragma unroll
        for (int u = 0; u < UN; ++u)
#pragma unroll
            for (int t = 0; t < MR; ++t)
#pragma unroll
                for (int c = 0; c < MC; ++c)
                    acc[t][c] = ks_mma(a[u][t], b[u][c], acc[t][c]);
    }
    ks_epilogue<MR, MC>(acc, g0, lcw, r, h, B, ncols, nlc, out, out_stride);
}

// Four-row-tile keyswitch with both operands staged by LDS-DMA (global_load_lds, 16 B per
// lane, no VGPR staging) through a ring of NB stages of SK k-steps (round 3).  PMC at 512
// gates of a register-staged version (digit tiles shared through LDS): 70 % of wave cycles
// parked on memory waits, the MFMA pipes 16 % busy -- each wave kept only one or two k-steps
// of fragments in flight against the HBM / L2 latency (more registers for more in flight
// cost occupancy; sharing the digit tiles alone gained nothing).  Here
// NB - 1 stages are in flight per workgroup at no register cost.  Wave w moves row tile w
// of the digits and column tile w of the limbs; every wave reads the four digit tiles and
// its own limb tile from the stage.  One raw barrier per stage, a counted vmcnt (never 0
// in steady state) so the DMAs of later stages stay in flight across it.  512 / 254 gates:
// keyswitch 98-100 -> 89-90 / 62-64 -> 55-57 us (tools/ks_probe.py; SK 1 / NB 8, SK 2 /
// NB 5, SK 1 / NB 10 and 4, 8, 10 K slices all measured slower: profiles/r03/ab_ks_glds.log)
template <int N>
__device__ __forceinline__ void ks_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    // s_waitcnt simm16 (gfx9): vmcnt [3:0] + [15:14], expcnt [6:4] = 7, lgkmcnt [11:8] = 15 (no wait)
    __builtin_amdgcn_s_waitcnt((N & 15) | (((N >> 4) & 3) << 14) | (7 << 4) | (15 << 8));
}
// wait until at most `after` stages of L DMAs each remain in flight (after <= A)
template <int L, int A>
__device__ __forceinline__ void ks_wait_after(int after) {
    if constexpr (A > 0) {
        if (after >= A) {
            ks_wait_vm<A * L>();
            return;
        }
        ks_wait_after<L, A - 1>(after);
    } else {
        ks_wait_vm<0>();
    }
}
template <int SK, int NB>
__global__ void __launch_bounds__(256)
k_ks_glds(const int8_t* __restrict__ dig, const int8_t* __restrict__ kl, int B, int KD, int ncols, int nlc,
          unsigned long long* __restrict__ out, int out_stride, int GX, int GY, int GZ, int xcd) {
    constexpr int MR = 4, L = 2 * SK;  // DMAs per wave per stage
    static_assert(NB >= 2 && (NB - 2) * 2 * SK < 64, "ring depth");
    __shared__ v4i_t ring[NB][2][4][SK][64];  // [stage][digits, limbs][tile][k-step][lane]
    KsTile tile;
    if (!ks_tile((int)blockIdx.x, GX, GY, GZ, xcd, tile)) return;  // padding workgroup (uniform)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int g0 = tile.x * 32 * MR;
    const int lcw = (tile.y * 4 + w) * 32;  // this wave's limb-column tile (past nlc: computed, dropped)
    const int kspan = KD / GZ, kb = tile.z * kspan, KT = KD / 32;
    const int8_t* ap = dig + ((size_t)((g0 >> 5) + w) * KT * 64 + lane) * 16 + (size_t)kb * 32;
    const int8_t* bp = kl + ((size_t)(min(lcw, nlc - 32) >> 5) * KT * 64 + lane) * 16 + (size_t)kb * 32;
    const int S = kspan / (32 * SK);  // kspan is a multiple of 256 (host)
    auto issue = [&](int st) {
        const int buf = st % NB;
#pragma unroll
        for (int u = 0; u < SK; ++u) {
            const size_t off = (size_t)(st * SK + u) * 32 * 32;
            __builtin_amdgcn_global_load_lds((const void*)(ap + off),
                                             (__attribute__((address_space(3))) void*)&ring[buf][0][w][u][0], 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(bp + off),
                                             (__attribute__((address_space(3))) void*)&ring[buf][1][w][u][0], 16, 0, 0);
        }
    };
    v16i_t acc[MR][1];
#pragma unroll
    for (int t = 0; t < MR; ++t) acc[t][0] = v16i_t{0};
#pragma unroll
    for (int st = 0; st < NB - 1; ++st)
        if (st < S) issue(st);
    for (int s = 0; s < S; ++s) {
        // this wave's DMAs of stage s have landed once at most those of the stages after it remain
        ks_wait_after<L, NB - 2>(min(NB - 2, S - 1 - s));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's stage s landed; stage s - 1's buffer read by all
        asm volatile("" ::: "memory");
        if (s + NB - 1 < S) issue(s + NB - 1);  // into stage s - 1's buffer
        const int cur = s % NB;
        v4i_t a[SK][MR], b[SK];
#pragma unroll
        for (int u = 0; u < SK; ++u) {
            b[u] = ring[cur][1][w][u][lane];
#pragma unroll
            for (int t = 0; t < MR; ++t) a[u][t] = ring[cur][0][t][u][lane];
        }
#pragma unroll
        for (int u = 0; u < SK; ++u)
#pragma unroll
            for (int t = 0; t < MR; ++t) acc[t][0] = ks_mma(a[u][t], b[u], acc[t][0]);
    }
    // Epilogue through LDS (the ring is free once every wave has passed the last stage): wave w
    // stores its 128 x 32 tile of i32 limb sums row-major ([row][limb column], 128 B rows,
    // conflict-free b32 stores), then lane L reads KSK column L & 3 of rows (L >> 2) + 16 j,
    // its 8 limbs as two b128 reads, recombines them in registers and subtracts the column with
    // one atomic: 8 atomics per lane, 16 rows x 4 adjacent columns per instruction (against 64
    // values x three 64-bit DPP rounds per lane in ks_epilogue)
    __syncthreads();
    if (lcw >= nlc) return;  // whole wave (no barrier below)
    int* tl = (int*)&ring[0][0][0][0][0] + w * 128 * 32;
#pragma unroll
    for (int t = 0; t < MR; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) tl[(32 * t + (i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[t][0][i];
    const int c = lane & 3, col = (lcw >> 3) + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int row = (lane >> 2) + 16 * j, g = g0 + row;
        const v4i_t lo = *(const v4i_t*)(tl + row * 32 + 8 * c), hi = *(const v4i_t*)(tl + row * 32 + 8 * c + 4);
        uint64_t v = 0;
#pragma unroll
        for (int l = 0; l < 4; ++l) v += ((uint64_t)(int64_t)lo[l] << (8 * l)) + ((uint64_t)(int64_t)hi[l] << (8 * l + 32));
        if (g < B && col < ncols && v != 0) atomicAdd(&out[(size_t)g * out_stride + col], (unsigned long long)(0 - v));
    }
}

// KSK (u64 [k][t], t <= n) -> balanced byte limbs in fragment order, limb l of column t at
// limb column ks_limb_col(t, l)
__global__ void __launch_bounds__(256) k_ksk_limbs(const uint64_t* __restrict__ ksk, int KD, int ncols, int nlc,
                                                   int8_t* __restrict__ kl) {
    const int KT = KD / 32;
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int t = blockIdx.y;
    if (k >= KD) return;
    uint64_t x = t < ncols ? ksk[(size_t)k * ncols + t] : 0;
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        int v = (int)(x & 255);
        x >>= 8;
        if (v >= 128) {
            v -= 256;
            x += 1;
        }
        const int lc = ks_limb_col(t, l);
        if (lc < nlc) kl[ks_frag(lc, k, KT)] = (int8_t)v;
    }
}

// linear combination into a slot (no bootstrap): NOT of a boolean, a match's final
// affine map.  The gate travels as a kernel argument (no staging copy before the launch).
__global__ void __launch_bounds__(256) k_linear(const DevGate gg, uint64_t* __restrict__ arena, int slot_stride,
                                                int len) {
    uint64_t* out = arena + (size_t)gg.out_slot[0] * slot_stride;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < len; t += gridDim.x * 256) {
        uint64_t v = (t == len - 1) ? ((uint64_t)(int64_t)gg.offset << (DELTA_LOG - 1)) : 0;
        for (int q = 0; q < gg.n_in; ++q) v += (uint64_t)(int64_t)gg.in_w[q] * arena[(size_t)gg.in_slot[q] * slot_stride + t];
        out[t] = v;
    }
}

// ================================================================== host side
#define STREAM ((hipStream_t)cur_stream())

template <int N, int K, int E>
static void set_smem_attr() {
    HIP_CHECK(hipFuncSetAttribute((const void*)k_blind_rotate<N, K, E>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)br_smem_bytes<N, K, E>()));
    HIP_CHECK(hipFuncSetAttribute((const void*)k_bsk_to_ntt<N, K, E>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)br_smem_bytes<N, K, E>()));
}

static bool supported(const Params& p) {
    if (p.ring == FR_RING_FFT) return (p.N == 2048 && p.k == 1) || (p.N == 1024 && p.k == 2);
    return (p.N == 2048 && p.k == 1) || (p.N == 1024 && p.k == 2) || (p.N == 1024 && p.k == 1);
}

// run `body` with compile-time (N, K, E) matching the runtime parameters
template <class F>
static void dispatch(const Params& p, int E, F&& body) {
    auto pick = [&](auto n, auto k, auto e) {
        if (p.N == decltype(n)::value && p.k == decltype(k)::value && E == decltype(e)::value) {
            body(n, k, e);
            return true;
        }
        return false;
    };
    using I2048 = std::integral_constant<int, 2048>;
    using I1024 = std::integral_constant<int, 1024>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using E8 = std::integral_constant<int, 8>;
    using E16 = std::integral_constant<int, 16>;
    if (pick(I2048{}, I1{}, E16{}) || pick(I2048{}, I1{}, E8{})) return;
    if (pick(I1024{}, I2{}, E16{}) || pick(I1024{}, I2{}, E8{})) return;
    if (pick(I1024{}, I1{}, E16{}) || pick(I1024{}, I1{}, E8{})) return;
    throw Error(FR_ERR_INVALID, "device: no kernel variant for (N, k, E)");
}

Device::Device(const Params& p, int device) : p_(p), dev_(device) {
    if (!supported(p)) throw Error(FR_ERR_INVALID, "device: unsupported (k, N)");
    if (p.ks_base_log != 3 || p.ks_level != 5 || p.pbs_base_log != 23 || p.pbs_level != 1)
        throw Error(FR_ERR_INVALID, "device: only KS 2^3x5 and PBS 2^23x1 are compiled");
    if (p.n > 1024) throw Error(FR_ERR_INVALID, "device: n > 1024");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0)
        throw Error(FR_ERR_NO_DEVICE, "no usable HIP device " + std::to_string(device));
    HIP_CHECK(hipSetDevice(device));
    hipStream_t s;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    stream_ = s;
    for (auto& e : ev_) {
        hipEvent_t ev;
        HIP_CHECK(hipEventCreate(&ev));
        e = ev;
    }
    for (auto* evs : {&stage_ev_, &cmap_ev_})
        for (auto& e : *evs) {
            hipEvent_t ev;
            HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIP_CHECK(hipEventRecord(ev, s));  // complete before first use
            e = ev;
        }
    // unrolled (k = 1) kernels keep three GGSW rows in registers: E = 8 only
    if (p.bsk_unroll() == 2) e_ = e_small_ = 8;
    if (const char* ev = std::getenv("FR_LANE_ELEMS")) e_ = std::atoi(ev);
    if (const char* ev = std::getenv("FR_SMALL_LANE_ELEMS")) e_small_ = std::atoi(ev);
    if (const char* ev = std::getenv("FR_SMALL_BATCH")) small_batch_ = (size_t)std::atol(ev);
    if (const char* ev = std::getenv("FR_KS_MFMA")) ks_mfma_ = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("FR_KS_MR4_MIN")) ks_mr4_min_ = (size_t)std::atol(ev);
    if (const char* ev = std::getenv("FR_KS_MC")) ks_mc_ = std::atoi(ev);
    if (const char* ev = std::getenv("FR_KS_SPLIT")) ks_split_ = std::atoi(ev);
    if (const char* ev = std::getenv("FR_TIMER_CHAIN")) timer_chain_ = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("FR_KS_XCD")) ks_xcd_ = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("FR_KS_LDS")) ks_lds_ = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("FR_KS_DIG16")) ks_dig16_ = std::atoi(ev) != 0;
    if ((e_ != 8 && e_ != 16) || (e_small_ != 8 && e_small_ != 16))
        throw Error(FR_ERR_INVALID, "FR_LANE_ELEMS / FR_SMALL_LANE_ELEMS must be 8 or 16");
    for (int e : {8, 16})
        dispatch(p_, e, [&](auto n, auto k, auto ec) { set_smem_attr<decltype(n)::value, decltype(k)::value, decltype(ec)::value>(); });
    // Montgomery-form forward twiddles, per prime: zeta_q[k] * 2^32 mod p_q
    NttTables T(p.N);
    std::vector<uint32_t> tw(2 * (size_t)p.N);
    for (int q = 0; q < 2; ++q)
        for (int i = 0; i < p.N; ++i) tw[(size_t)q * p.N + i] = (uint32_t)(((uint64_t)T.zeta[q][i] << 32) % rns::prime(q));
    HIP_CHECK(hipMalloc(&d_tw_, 4 * tw.size()));
    HIP_CHECK(hipMemcpy(d_tw_, tw.data(), 4 * tw.size(), hipMemcpyHostToDevice));
    if (p.ring == FR_RING_FFT) init_fft();
    ensure_arena(1024);
    ensure_batch(1024);
}

Device::~Device() {
    (void)hipSetDevice(dev_);
    if (lane_ != 0) leave_lane();
    for (auto& l : lanes_) {
        if (l.stream) (void)hipStreamSynchronize((hipStream_t)l.stream);
        free_lane(l);
    }
    lanes_.clear();
    if (main_ev_) (void)hipEventDestroy((hipEvent_t)main_ev_);
    if (stream_) (void)hipStreamSynchronize((hipStream_t)stream_);
    (void)hipFree(d_ksk_);
    (void)hipFree(d_tbsk_);
    (void)hipFree(d_kl_);
    (void)hipFree(d_dig_);
    (void)hipFree(d_bsk_);
    (void)hipFree(d_tw_);
    free_fft();
    (void)hipFree(d_arena_);
    (void)hipFree(d_gates_);
    (void)hipFree(d_ks_);
    (void)hipFree(d_slot_list_);
    for (auto* h : h_stage_)
        if (h) (void)hipHostFree(h);
    for (auto* e : stage_ev_)
        if (e) (void)hipEventDestroy((hipEvent_t)e);
    for (auto* e : cmap_ev_)
        if (e) (void)hipEventDestroy((hipEvent_t)e);
    (void)hipFree(d_cmap_);
    for (auto* h : h_cmap_)
        if (h) (void)hipHostFree(h);
    for (auto& t : pending_)
        for (auto* e : t.ev) (void)hipEventDestroy((hipEvent_t)e);
    for (auto* e : event_pool_) (void)hipEventDestroy((hipEvent_t)e);
    for (auto e : ev_)
        if (e) (void)hipEventDestroy((hipEvent_t)e);
    if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

// ---------------------------------------------------------------- lanes
void Device::swap_lane(LaneState& l) {
    std::swap(stream_, l.stream);
    std::swap(d_ks_, l.d_ks);
    std::swap(batch_cap_, l.batch_cap);
    std::swap(d_dig_, l.d_dig);
    std::swap(dig_cap_, l.dig_cap);
    std::swap(d_cmap_, l.d_cmap);
    std::swap(h_cmap_, l.h_cmap);
    std::swap(cmap_ev_, l.cmap_ev);
    std::swap(cmap_cap_, l.cmap_cap);
    std::swap(cmap_n_, l.cmap_n);
    std::swap(cmap_stage_, l.cmap_stage);
}
void Device::free_lane(LaneState& l) {
    (void)hipFree(l.d_ks);
    (void)hipFree(l.d_dig);
    (void)hipFree(l.d_cmap);
    for (auto* h : l.h_cmap)
        if (h) (void)hipHostFree(h);
    for (auto* e : l.cmap_ev)
        if (e) (void)hipEventDestroy((hipEvent_t)e);
    if (l.done_ev) (void)hipEventDestroy((hipEvent_t)l.done_ev);
    if (l.stream) (void)hipStreamDestroy((hipStream_t)l.stream);
    l = LaneState{};
}
void Device::set_lanes(int n) {
    if (n < 1 || n > 8) throw Error(FR_ERR_INVALID, "lanes: 1..8");
    if (lane_ != 0) throw Error(FR_ERR_INVALID, "lanes: changed inside a lane");
    sync_all();
    // n >= 2: n lanes besides lane 0 (matches go to them only: a match on lane 0 would wait
    // for the other lanes at its first launch)
    const int extra = n >= 2 ? n : 0;
    while ((int)lanes_.size() > extra) {
        free_lane(lanes_.back());
        lanes_.pop_back();
    }
    if (!main_ev_ && extra) {
        hipEvent_t ev;
        HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        main_ev_ = ev;
    }
    while ((int)lanes_.size() < extra) {
        LaneState l;
        hipStream_t st;
        HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        l.stream = st;
        for (auto*& e : l.cmap_ev) {
            hipEvent_t ev;
            HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIP_CHECK(hipEventRecord(ev, st));  // complete before first use
            e = ev;
        }
        hipEvent_t dv;
        HIP_CHECK(hipEventCreateWithFlags(&dv, hipEventDisableTiming));
        l.done_ev = dv;
        lanes_.push_back(l);
        // the lane's keyswitch scratch at the main lane's size (ensure_batch on entry grows it)
        const int i = (int)lanes_.size();
        enter_lane(i);
        ensure_batch(1024);
        leave_lane();
    }
}
void Device::enter_lane(int i) {
    if (lane_ != 0) throw Error(FR_ERR_INVALID, "lanes: already inside a lane");
    if (i <= 0) return;
    if (i > (int)lanes_.size()) throw Error(FR_ERR_INVALID, "lanes: no such lane");
    // the lane waits for lane 0's own work so far -- not for the other lanes (no join here:
    // that would chain every lane behind the previous one); lane 0 waited for the lanes at
    // its last operation, so their results that operation consumed are covered too
    HIP_CHECK(hipEventRecord((hipEvent_t)main_ev_, (hipStream_t)stream_));
    swap_lane(lanes_[i - 1]);
    lane_ = i;
    HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream_, (hipEvent_t)main_ev_, 0));
}
void Device::leave_lane() {
    if (lane_ == 0) return;
    LaneState& l = lanes_[lane_ - 1];
    HIP_CHECK(hipEventRecord((hipEvent_t)l.done_ev, (hipStream_t)stream_));
    swap_lane(l);
    l.pending = true;
    lanes_pending_ = true;
    lanes_unsynced_ = true;
    lane_ = 0;
}
void Device::join_lanes() {
    if (!lanes_pending_ || lane_ != 0) return;
    for (auto& l : lanes_)
        if (l.pending) {
            HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream_, (hipEvent_t)l.done_ev, 0));
            l.pending = false;
        }
    lanes_pending_ = false;
}
void* Device::cur_stream() {
    if (lane_ == 0 && lanes_pending_) join_lanes();
    return stream_;
}
void Device::sync_all() {
    HIP_CHECK(hipStreamSynchronize((hipStream_t)stream_));
    for (auto& l : lanes_)
        if (l.stream) HIP_CHECK(hipStreamSynchronize((hipStream_t)l.stream));
    if (lane_ == 0) {
        for (auto& l : lanes_) l.pending = false;
        lanes_pending_ = false;
    }
    lanes_unsynced_ = false;
    free_slots_.insert(free_slots_.end(), deferred_free_.begin(), deferred_free_.end());
    deferred_free_.clear();
}

std::string Device::info() const {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, dev_);
    std::ostringstream o;
    o << prop.name << " " << prop.gcnArchName << " CUs=" << prop.multiProcessorCount;
    if (p_.ring == FR_RING_FFT) o << " ring=fft E=" << fft_e_ << " latency<=" << fft_small_;
    else o << " ring=rns E=" << e_;
    return o.str();
}

void Device::ensure_arena(size_t slots) {
    if (slots <= arena_cap_) return;
    size_t cap = arena_cap_ ? arena_cap_ : 1024;
    while (cap < slots) cap *= 2;
    uint64_t* nb = nullptr;
    HIP_CHECK(hipMalloc(&nb, (size_t)8 * p_.slot_stride() * cap));
    if (d_arena_) {
        sync_all();  // no launch of any lane may still use the old arena
        HIP_CHECK(hipMemcpyAsync(nb, d_arena_, (size_t)8 * p_.slot_stride() * arena_cap_, hipMemcpyDeviceToDevice, STREAM));
        HIP_CHECK(hipStreamSynchronize(STREAM));
        HIP_CHECK(hipFree(d_arena_));
    }
    d_arena_ = nb;
    arena_cap_ = cap;
}

void Device::ensure_digits(size_t rows) {
    if (rows <= dig_cap_) return;
    size_t cap = dig_cap_ ? dig_cap_ : 1024;
    while (cap < rows) cap *= 2;
    HIP_CHECK(hipStreamSynchronize(STREAM));
    (void)hipFree(d_dig_);
    HIP_CHECK(hipMalloc(&d_dig_, cap * (size_t)p_.big() * p_.ks_level));
    dig_cap_ = cap;
}

void Device::ensure_batch(size_t n) {
    if (n <= batch_cap_) return;
    size_t cap = batch_cap_ ? batch_cap_ : 1024;
    while (cap < n) cap *= 2;
    HIP_CHECK(hipStreamSynchronize(STREAM));
    (void)hipFree(d_ks_);
    if (lane_ == 0) {  // the gate staging ring belongs to lane 0 (lanes run resident plans only)
        (void)hipFree(d_gates_);
        for (auto& h : h_stage_) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
        }
        HIP_CHECK(hipMalloc(&d_gates_, sizeof(DevGate) * cap));
        for (auto& h : h_stage_) HIP_CHECK(hipHostMalloc(&h, sizeof(DevGate) * cap));
    }
    HIP_CHECK(hipMalloc(&d_ks_, (size_t)8 * p_.ks_stride() * cap));
    batch_cap_ = cap;
}

int Device::alloc_slot() {
    if (!free_slots_.empty()) {
        int s = free_slots_.back();
        free_slots_.pop_back();
        return s;
    }
    ensure_arena(next_slot_ + 1);
    return (int)next_slot_++;
}
void Device::free_slot(int s) {
    if (s < 0) return;
    // a lane may still read or write it: recycled after the next host sync of every lane
    if (lanes_unsynced_ || lane_ != 0) {
        deferred_free_.push_back(s);
        // a serving loop that never downloads: recycle in bulk rather than grow the arena
        if (deferred_free_.size() >= (size_t)1 << 16) sync_all();
    } else {
        free_slots_.push_back(s);
    }
}

// packed copies between arena slots and a device buffer of the caller (the
// multi-rank exchange of a level's outputs: fr_shard_export / fr_shard_import):
// one workgroup per LWE, lwe_len u64 each, coalesced
__global__ void __launch_bounds__(256) k_slots_to_buf(const uint64_t* __restrict__ arena, int stride,
                                                      const int* __restrict__ slots, int len, uint64_t* __restrict__ buf) {
    const uint64_t* s = arena + (size_t)slots[blockIdx.x] * stride;
    uint64_t* d = buf + (size_t)blockIdx.x * len;
    for (int c = threadIdx.x; c < len; c += 256) d[c] = s[c];
}
__global__ void __launch_bounds__(256) k_buf_to_slots(const uint64_t* __restrict__ buf, int len,
                                                      const int* __restrict__ slots, int stride, uint64_t* __restrict__ arena) {
    const uint64_t* s = buf + (size_t)blockIdx.x * len;
    uint64_t* d = arena + (size_t)slots[blockIdx.x] * stride;
    for (int c = threadIdx.x; c < len; c += 256) d[c] = s[c];
}
struct SlotArgs {
    int s[16];
};
__global__ void __launch_bounds__(256) k_slots_to_buf_arg(const uint64_t* __restrict__ arena, int stride, SlotArgs sl,
                                                          int len, uint64_t* __restrict__ buf) {
    const uint64_t* s = arena + (size_t)sl.s[blockIdx.x] * stride;
    uint64_t* d = buf + (size_t)blockIdx.x * len;
    for (int c = threadIdx.x; c < len; c += 256) d[c] = s[c];
}
void Device::slots_to_device_async(const int* slots, size_t n, uint64_t* dst) {
    if (!n) return;
    if (n > 16) throw Error(FR_ERR_INVALID, "slots_to_device_async: at most 16 slots");
    SlotArgs a{};
    for (size_t i = 0; i < n; ++i) {
        if (slots[i] < 0 || (size_t)slots[i] >= next_slot_) throw Error(FR_ERR_INVALID, "slot list: slot out of range");
        a.s[i] = slots[i];
    }
    k_slots_to_buf_arg<<<(unsigned)n, 256, 0, STREAM>>>(d_arena_, p_.slot_stride(), a, p_.lwe_len(), dst);
    HIP_CHECK(hipGetLastError());
}
void Device::stage_slot_list(const int* slots, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (slots[i] < 0 || (size_t)slots[i] >= next_slot_) throw Error(FR_ERR_INVALID, "slot list: slot out of range");
    if (n > slot_list_cap_) {
        HIP_CHECK(hipStreamSynchronize(STREAM));
        (void)hipFree(d_slot_list_);
        d_slot_list_ = nullptr;
        slot_list_cap_ = std::max<size_t>(n, 1024);
        HIP_CHECK(hipMalloc(&d_slot_list_, 4 * slot_list_cap_));
    }
    HIP_CHECK(hipMemcpyAsync(d_slot_list_, slots, 4 * n, hipMemcpyHostToDevice, STREAM));
}
void Device::slots_to_device(const int* slots, size_t n, uint64_t* dst) {
    if (!n) return;
    stage_slot_list(slots, n);
    k_slots_to_buf<<<(unsigned)n, 256, 0, STREAM>>>(d_arena_, p_.slot_stride(), d_slot_list_, p_.lwe_len(), dst);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(STREAM));  // the caller's stream may read dst now
}
void Device::device_to_slots(const int* slots, size_t n, const uint64_t* src) {
    if (!n) return;
    stage_slot_list(slots, n);
    k_buf_to_slots<<<(unsigned)n, 256, 0, STREAM>>>(src, p_.lwe_len(), d_slot_list_, p_.slot_stride(), d_arena_);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(STREAM));  // the caller may reuse src now
}

void Device::write_slots(const int* slots, size_t n, const uint64_t* host) {
    const int L = p_.lwe_len(), S = p_.slot_stride();
    for (size_t i = 0; i < n; ++i)
        HIP_CHECK(hipMemcpyAsync(d_arena_ + (size_t)slots[i] * S, host + i * L, 8 * (size_t)L, hipMemcpyHostToDevice, STREAM));
    HIP_CHECK(hipStreamSynchronize(STREAM));
}
void Device::read_slot(int slot, uint64_t* host) {
    HIP_CHECK(hipMemcpyAsync(host, d_arena_ + (size_t)slot * p_.slot_stride(), 8 * (size_t)p_.lwe_len(),
                             hipMemcpyDeviceToHost, STREAM));
    sync_all();
}
void Device::zero_slot(int slot) {
    HIP_CHECK(hipMemsetAsync(d_arena_ + (size_t)slot * p_.slot_stride(), 0, 8 * (size_t)p_.lwe_len(), STREAM));
}

// byte-limb form of the KSK for the MFMA keyswitch
void Device::build_ksk_limbs() {
    const int KD = p_.big() * p_.ks_level, ncols = p_.n + 1;
    const int nlc = ((ncols * 8 + 127) / 128) * 128;  // whole 4-wave column groups
    (void)hipFree(d_kl_);
    d_kl_ = nullptr;
    HIP_CHECK(hipMalloc(&d_kl_, (size_t)nlc * KD));
    HIP_CHECK(hipMemsetAsync(d_kl_, 0, (size_t)nlc * KD, STREAM));
    k_ksk_limbs<<<dim3((unsigned)((KD + 255) / 256), (unsigned)(nlc / 8)), 256, 0, STREAM>>>(d_ksk_, KD, ncols, nlc,
                                                                                          d_kl_);
    HIP_CHECK(hipGetLastError());
    kl_cols_ = nlc;
}

void Device::upload_keys(const std::vector<uint64_t>& ksk, const std::vector<uint64_t>& bsk) {
    if (ksk.size() != (size_t)p_.big() * p_.ks_level * (p_.n + 1)) throw Error(FR_ERR_INVALID, "ksk size");
    if (bsk.size() != p_.bsk_len()) throw Error(FR_ERR_INVALID, "bsk size");
    // every queued launch of every lane that reads the old keys has finished before they go
    HIP_CHECK(hipDeviceSynchronize());
    (void)hipFree(d_ksk_);
    (void)hipFree(d_bsk_);
    d_ksk_ = nullptr;
    d_bsk_ = nullptr;
    HIP_CHECK(hipMalloc(&d_ksk_, 8 * ksk.size()));
    HIP_CHECK(hipMemcpy(d_ksk_, ksk.data(), 8 * ksk.size(), hipMemcpyHostToDevice));
    (void)hipFree(d_tbsk_);  // host-generated keys: export reads the host copy
    d_tbsk_ = nullptr;
    build_ksk_limbs();
    if (p_.ring == FR_RING_FFT) {
        upload_fft_bsk(bsk);
        return;
    }
    uint64_t* coef = nullptr;
    HIP_CHECK(hipMalloc(&coef, 8 * bsk.size()));
    HIP_CHECK(hipMemcpy(coef, bsk.data(), 8 * bsk.size(), hipMemcpyHostToDevice));
    HIP_CHECK(hipMalloc(&d_bsk_, 4 * 2 * bsk.size()));  // two u32 residues per coefficient
    // 1/N in Montgomery form per prime
    uint32_t ninv_r[2];
    for (int q = 0; q < 2; ++q) {
        const uint64_t pq = rns::prime(q);
        uint64_t inv = 1, b = (uint64_t)p_.N % pq, e = pq - 2;
        while (e) {
            if (e & 1) inv = inv * b % pq;
            b = b * b % pq;
            e >>= 1;
        }
        ninv_r[q] = (uint32_t)((inv << 32) % pq);
    }
    const int blocks = (int)p_.bsk_ggsw() * (p_.k + 1);
    dispatch(p_, e_, [&](auto n_, auto k_, auto e_c) {
        constexpr int N = decltype(n_)::value, K = decltype(k_)::value, E = decltype(e_c)::value;
        k_bsk_to_ntt<N, K, E><<<blocks, br_threads<N, K, E>(), br_smem_bytes<N, K, E>(), STREAM>>>(coef, d_tw_, ninv_r[0],
                                                                                                    ninv_r[1], d_bsk_);
    });
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(STREAM));
    HIP_CHECK(hipFree(coef));
}

void Device::launch_ks(const DevGate* d_gates, size_t n, uint64_t* d_ks, void* ev_start, void* ev_stop) {
    const hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
    if (ks_mfma_) {
        const int KD = p_.big() * p_.ks_level;
        if (KD % 256) throw Error(FR_ERR_INVALID, "MFMA keyswitch needs kN*ks_level % 256 == 0");
        const int MR = n >= ks_mr4_min_ ? 4 : 1;  // row tiles per wave
        const size_t bp = (n + 32 * MR - 1) / (32 * MR) * (32 * MR);
        ensure_digits(bp);
        if (KD % 16) throw Error(FR_ERR_INVALID, "MFMA keyswitch: digit rows must be whole 16-byte vectors");
        if (ks_dig16_ && p_.big() % 16 == 0)
            hipExtLaunchKernelGGL(k_ks_digits16<3, 5>, dim3((unsigned)bp), dim3(128), 0, STREAM, e0, nullptr, 0, d_gates,
                                  (int)n, (const uint64_t*)d_arena_, p_.slot_stride(), (const int*)d_cmap_, p_.big(),
                                  d_dig_, d_ks, p_.n, p_.ks_stride());
        else
            hipExtLaunchKernelGGL(k_ks_digits<3, 5>, dim3(8, (unsigned)bp), dim3(256), 0, STREAM, e0, nullptr, 0, d_gates,
                                  (int)n, (const uint64_t*)d_arena_, p_.slot_stride(), (const int*)d_cmap_, p_.big(),
                                  d_dig_, d_ks, p_.n, p_.ks_stride());
        HIP_CHECK(hipGetLastError());
        // column tiles per wave: 1 (FR_KS_MC=2 shares each digit fragment between two; with
        // fragment-ordered operands that no longer pays: 512 gates 121 -> 103 us at 1)
        const int MC = MR == 4 && ks_mc_ == 2 ? 2 : 1;
        // K slices (partial sums meet in 64-bit atomics, so more slices cost atomic traffic, and
        // every slice its epilogue): 8 for one row tile per wave (1-17 gates ~30 us); four row
        // tiles (k_ks_glds): 5 up to 256 gates, 2 up to 512, then 1 (profiles/r03/ab_ks_glds.log:
        // 254 gates 55 us at 4-5 against 60 at 2; 512: 77 at 2 against 86-89 at 4-5; 1024 /
        // 2048: 125 / 231 at 1 against 130 / 234 at 2); a divisor of KD / 256
        const int gx = (int)(bp / (32 * MR));
        int split = MR == 1 ? 8 : gx <= 2 ? 5 : gx <= 4 ? 2 : 1;
        while ((KD / 256) % split) --split;
        if (ks_split_ > 0 && (KD / 256) % ks_split_ == 0) split = ks_split_;
        const int GX = gx, GY = (kl_cols_ + 128 * MC - 1) / (128 * MC), GZ = split;
        const dim3 grid((unsigned)ks_grid_blocks(GX, GY, GZ, ks_xcd_));
        if (MR == 4 && MC == 1 && ks_lds_)
            hipExtLaunchKernelGGL(k_ks_glds<FR_KS_SK, FR_KS_NB>, grid, dim3(256), 0, STREAM, nullptr, e1, 0,
                                  (const int8_t*)d_dig_, (const int8_t*)d_kl_, (int)n, KD, p_.n + 1, kl_cols_,
                                  (unsigned long long*)d_ks, p_.ks_stride(), GX, GY, GZ, ks_xcd_);
        else if (MR == 4 && MC == 2)
            hipExtLaunchKernelGGL(k_ks_mfma<4, 2>, grid, dim3(256), 0, STREAM, nullptr, e1, 0, (const int8_t*)d_dig_,
                                  (const int8_t*)d_kl_, (int)n, KD, p_.n + 1, kl_cols_, (unsigned long long*)d_ks,
                                  p_.ks_stride(), GX, GY, GZ, ks_xcd_);
        else if (MR == 4)
            hipExtLaunchKernelGGL(k_ks_mfma<4, 1>, grid, dim3(256), 0, STREAM, nullptr, e1, 0, (const int8_t*)d_dig_,
                                  (const int8_t*)d_kl_, (int)n, KD, p_.n + 1, kl_cols_, (unsigned long long*)d_ks,
                                  p_.ks_stride(), GX, GY, GZ, ks_xcd_);
        else
            hipExtLaunchKernelGGL(k_ks_mfma<1, 1>, grid, dim3(256), 0, STREAM, nullptr, e1, 0, (const int8_t*)d_dig_,
                                  (const int8_t*)d_kl_, (int)n, KD, p_.n + 1, kl_cols_, (unsigned long long*)d_ks,
                                  p_.ks_stride(), GX, GY, GZ, ks_xcd_);
        HIP_CHECK(hipGetLastError());
        return;
    }
    const int btiles = (int)((n + KS_BT - 1) / KS_BT);
    const int ctiles = (p_.n + 1 + KS_CT - 1) / KS_CT;
    const int chunks = (p_.big() + KS_CH - 1) / KS_CH;
    // enough workgroups to fill 256 CUs several times over, in whole chunks
    int splits = (2048 + btiles * ctiles - 1) / (btiles * ctiles);
    splits = std::max(1, std::min(splits, chunks));
    const int per = (chunks + splits - 1) / splits;
    splits = (chunks + per - 1) / per;
    if (splits > 1) HIP_CHECK(hipMemsetAsync(d_ks, 0, (size_t)8 * p_.ks_stride() * n, STREAM));
    dim3 grid((unsigned)btiles, (unsigned)ctiles, (unsigned)splits);
    hipExtLaunchKernelGGL(k_lincomb_keyswitch<3, 5>, grid, dim3(256), 0, STREAM, e0, e1, 0, d_gates, (int)n,
                          (const uint64_t*)d_arena_, p_.slot_stride(), (const int*)d_cmap_, (const uint64_t*)d_ksk_, p_.n,
                          p_.big(), per, (unsigned long long*)d_ks, p_.ks_stride());
    HIP_CHECK(hipGetLastError());
}

bool Device::latency_shape(size_t n) const { return n <= (p_.ring == FR_RING_FFT ? fft_small_ : small_batch_); }
bool Device::pair_shape(size_t n) const { return p_.ring == FR_RING_FFT && !latency_shape(n) && n <= fft_pair_; }

void Device::launch_br(const DevGate* d_gates, const uint64_t* d_ks, size_t n, void* ev_start, void* ev_stop) {
    if (p_.ring == FR_RING_FFT) {
        launch_br_fft(d_gates, d_ks, n, stream_, ev_start, ev_stop);
        return;
    }
    // small levels (at most one bootstrap per CU): more lanes per bootstrap for latency
    const int E = n <= small_batch_ ? e_small_ : e_;
    dispatch(p_, E, [&](auto n_, auto k_, auto e_c) {
        constexpr int N = decltype(n_)::value, K = decltype(k_)::value, E = decltype(e_c)::value;
        hipExtLaunchKernelGGL(k_blind_rotate<N, K, E>, dim3((unsigned)n), dim3(br_threads<N, K, E>()),
                              (uint32_t)br_smem_bytes<N, K, E>(), STREAM, (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0,
                              d_ks, p_.ks_stride(), p_.n, d_gates, (const uint32_t*)d_bsk_, (const uint32_t*)d_tw_,
                              d_arena_, p_.slot_stride());
    });
    HIP_CHECK(hipGetLastError());
}

void Device::validate_gates(const DevGate* gates, size_t n, size_t n_refs) const {
    for (size_t i = 0; i < n; ++i) {
        const DevGate& g = gates[i];
        if (g.n_in < 0 || g.n_in > 16 || g.n_out < 1 || g.n_out > MAX_OUT || g.direct < 0 || g.direct > 2 ||
            (g.direct && g.n_out != 1))
            throw Error(FR_ERR_INVALID, "device gate: bad descriptor");
        for (int f = 0; f < g.n_out; ++f)
            if (g.out_slot[f] < 0 || (size_t)g.out_slot[f] >= next_slot_) throw Error(FR_ERR_INVALID, "device gate: bad output slot");
        for (int q = 0; q < g.n_in; ++q) {
            const int s = g.in_slot[q];
            if (s >= 0 ? (size_t)s >= next_slot_ : (size_t)(-1 - (int64_t)s) >= n_refs)
                throw Error(FR_ERR_INVALID, "device gate: bad input slot");
        }
    }
}

void Device::bind_content(const int* cmap, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (cmap[i] < -1 || (cmap[i] >= 0 && (size_t)cmap[i] >= next_slot_))
            throw Error(FR_ERR_INVALID, "content map: slot out of range");
    if (n > cmap_cap_) {
        HIP_CHECK(hipStreamSynchronize(STREAM));  // no launch may still read the old map
        (void)hipFree(d_cmap_);
        d_cmap_ = nullptr;
        for (auto& h : h_cmap_) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
        }
        size_t cap = cmap_cap_ ? cmap_cap_ : 4096;
        while (cap < n) cap *= 2;
        HIP_CHECK(hipMalloc(&d_cmap_, 4 * cap));
        for (auto& h : h_cmap_) HIP_CHECK(hipHostMalloc(&h, 4 * cap));
        cmap_cap_ = cap;
    }
    // the map bound last is still in place (a replay of the same content): nothing to copy
    if (n == cmap_n_ && n && std::memcmp(h_cmap_[cmap_stage_], cmap, 4 * n) == 0) return;
    cmap_stage_ ^= 1;
    // the pinned buffer is rewritten only after its previous copy completed
    HIP_CHECK(hipEventSynchronize((hipEvent_t)cmap_ev_[cmap_stage_]));
    std::memcpy(h_cmap_[cmap_stage_], cmap, 4 * n);
    if (n) HIP_CHECK(hipMemcpyAsync(d_cmap_, h_cmap_[cmap_stage_], 4 * n, hipMemcpyHostToDevice, STREAM));
    HIP_CHECK(hipEventRecord((hipEvent_t)cmap_ev_[cmap_stage_], STREAM));
    cmap_n_ = n;
}

void Device::run_level(const DevGate* gates, size_t n) {
    if (!n) return;
    if (!has_keys()) throw Error(FR_ERR_NO_KEY, "server key not uploaded");
    if (lane_ != 0) throw Error(FR_ERR_INVALID, "staged gate batches run on lane 0 only");
    validate_gates(gates, n);
    ensure_batch(n);
    // d_gates_ / d_ks_ are reused in stream order (this level's copy runs after
    // the previous level's kernels); only the host staging buffer needs a wait
    std::memcpy(stage_acquire(), gates, sizeof(DevGate) * n);
    stage_copy(n);
    launch_level(d_gates_, gates, n);
}

void Device::run_level_resident(const DevGate* d_gates, const DevGate* host, size_t n, size_t n_refs) {
    if (!n) return;
    if (!has_keys()) throw Error(FR_ERR_NO_KEY, "server key not uploaded");
    if (n_refs > cmap_n_) throw Error(FR_ERR_INVALID, "template plan: content map not bound");
    ensure_batch(n);
    launch_level(d_gates, host, n);
}

DevGate* Device::upload_gates(const DevGate* gates, size_t n, size_t n_refs) {
    validate_gates(gates, n, n_refs);
    DevGate* d = nullptr;
    HIP_CHECK(hipMalloc(&d, sizeof(DevGate) * std::max<size_t>(n, 1)));
    HIP_CHECK(hipMemcpy(d, gates, sizeof(DevGate) * n, hipMemcpyHostToDevice));
    return d;
}

void Device::free_gates(DevGate* d) {
    if (!d) return;
    HIP_CHECK(hipStreamSynchronize(STREAM));
    HIP_CHECK(hipFree(d));
}

void Device::launch_level(const DevGate* d_gates, const DevGate* host, size_t n) {
    PendingTimer t{};
    if (profiling_)
        for (auto& e : t.ev) e = take_event();
    // keyswitch events at level 2 only: two more event-stamped launches per level cost
    // ~30 us per /abc/ match (tools/match_probe.py).  Level 1 stamps stop events only: the
    // blind rotation runs from the keyswitch's end event to its own (the launch gap between
    // them, ~0 without a start event, counts as rotation time).  A start event on the BR
    // launch opened a ~6.6 us gap before it and the stop events ~4.7 us after it under the
    // kernel trace (profiles/r04/gaps/).
    t.chain = profiling_ == 1 && timer_chain_;
    if (profiling_ >= 2) launch_ks(d_gates, n, d_ks_, t.ev[0], t.ev[1]);
    else launch_ks(d_gates, n, d_ks_, nullptr, t.chain ? t.ev[1] : nullptr);
    launch_br(d_gates, d_ks_, n, t.chain ? nullptr : t.ev[2], t.ev[3]);
    HIP_CHECK(hipGetLastError());
    if (profiling_) {
        t.gates = n;
        t.lat = latency_shape(n);
        t.pair = pair_shape(n) && !fft_dual_;  // FR_FFT_DUAL launches: one bootstrap per workgroup
        t.ks = profiling_ >= 2;
        t.outs = 0;
        for (size_t i = 0; i < n; ++i) t.outs += host[i].n_out;
        pending_.push_back(t);
    }
}

DevGate* Device::stage_acquire() {
    stage_ ^= 1;
    HIP_CHECK(hipEventSynchronize((hipEvent_t)stage_ev_[stage_]));  // never-recorded events are complete
    return h_stage_[stage_];
}
void Device::stage_copy(size_t n) {
    HIP_CHECK(hipMemcpyAsync(d_gates_, h_stage_[stage_], sizeof(DevGate) * n, hipMemcpyHostToDevice, STREAM));
    HIP_CHECK(hipEventRecord((hipEvent_t)stage_ev_[stage_], STREAM));
}
void* Device::take_event() {
    if (!event_pool_.empty()) {
        void* e = event_pool_.back();
        event_pool_.pop_back();
        return e;
    }
    // timing-only events (read after a stream sync): a device-scope release instead of
    // the system-scope fence, so recording one between two launches costs no cache
    // writeback (with the default fence each record opened a ~5 us gap in the level chain)
    // (the first flag set this runtime accepts)
    hipEvent_t ev = nullptr;
    for (unsigned fl : {(unsigned)hipEventReleaseToDevice, (unsigned)hipEventDisableSystemFence, (unsigned)hipEventDefault})
        if (hipEventCreateWithFlags(&ev, fl) == hipSuccess) return ev;
        else (void)hipGetLastError();
    HIP_CHECK(hipEventCreate(&ev));
    return ev;
}
// KS / BR kernel times of the levels issued since the last sync (HIP events
// on the launch stream, read once the stream has drained)
void Device::resolve_timers() {
    for (auto& t : pending_) {
        float ks = 0, br = 0;
        if (t.ks) HIP_CHECK(hipEventElapsedTime(&ks, (hipEvent_t)t.ev[0], (hipEvent_t)t.ev[1]));
        HIP_CHECK(hipEventElapsedTime(&br, (hipEvent_t)t.ev[t.chain ? 1 : 2], (hipEvent_t)t.ev[3]));
        timers_.ks_ms += ks;
        timers_.br_ms += br;
        timers_.br_launches += 1;
        timers_.br_gates += t.gates;
        timers_.lut_outputs += t.outs;
        if (t.lat) {
            timers_.lat_br_ms += br;
            timers_.lat_launches += 1;
            timers_.lat_gates += t.gates;
        }
        if (t.pair) {
            timers_.pair_br_ms += br;
            timers_.pair_launches += 1;
            timers_.pair_gates += t.gates;
        }
        for (auto* e : t.ev) event_pool_.push_back(e);
    }
    pending_.clear();
}

void Device::run_linear(const DevGate& g) {
    k_linear<<<(p_.lwe_len() + 255) / 256, 256, 0, STREAM>>>(g, d_arena_, p_.slot_stride(), p_.lwe_len());
    HIP_CHECK(hipGetLastError());
}

void Device::sync() {
    sync_all();
    resolve_timers();
}

// ---------------------------------------------------------------- tests
void Device::keyswitch_host(const uint64_t* in, size_t count, uint64_t* out) {
    if (!has_keys()) throw Error(FR_ERR_NO_KEY, "server key not uploaded");
    HIP_CHECK(hipStreamSynchronize(STREAM));  // queued matches read d_ks_ / d_gates_ (blind_rotate_host)
    std::vector<int> slots(count);
    std::vector<DevGate> gates(count);
    for (size_t i = 0; i < count; ++i) slots[i] = alloc_slot();
    write_slots(slots.data(), count, in);
    for (size_t i = 0; i < count; ++i) {
        std::memset(&gates[i], 0, sizeof(DevGate));
        gates[i].n_in = 1;
        gates[i].in_slot[0] = slots[i];
        gates[i].in_w[0] = 1;
        gates[i].n_out = 1;
        gates[i].direct = JOB_DIRECT;
        gates[i].out_slot[0] = slots[i];
    }
    ensure_batch(count);
    HIP_CHECK(hipMemcpy(d_gates_, gates.data(), sizeof(DevGate) * count, hipMemcpyHostToDevice));
    launch_ks(d_gates_, count, d_ks_);
    HIP_CHECK(hipStreamSynchronize(STREAM));
    const int ks = p_.ks_stride();
    for (size_t i = 0; i < count; ++i)
        HIP_CHECK(hipMemcpy(out + i * (p_.n + 1), d_ks_ + i * ks, 8 * (size_t)(p_.n + 1), hipMemcpyDeviceToHost));
    for (int s : slots) free_slot(s);
}

void Device::blind_rotate_host(const uint64_t* ks_in, const uint8_t* luts, size_t count, uint64_t* out) {
    if (!has_keys()) throw Error(FR_ERR_NO_KEY, "server key not uploaded");
    // an asynchronous match may still read d_ks_ / d_gates_ on STREAM; the plain
    // copies below run on the null stream, which does not wait for a non-blocking one
    HIP_CHECK(hipStreamSynchronize(STREAM));
    ensure_batch(count);
    const int ks = p_.ks_stride();
    for (size_t i = 0; i < count; ++i)
        HIP_CHECK(hipMemcpy(d_ks_ + i * ks, ks_in + i * (p_.n + 1), 8 * (size_t)(p_.n + 1), hipMemcpyHostToDevice));
    std::vector<int> slots(count);
    std::vector<DevGate> gates(count);
    for (size_t i = 0; i < count; ++i) {
        slots[i] = alloc_slot();
        std::memset(&gates[i], 0, sizeof(DevGate));
        std::memcpy(gates[i].lut[0], luts + 16 * i, 16);
        gates[i].n_out = 1;
        gates[i].direct = JOB_DIRECT;
        gates[i].out_slot[0] = slots[i];
    }
    HIP_CHECK(hipMemcpy(d_gates_, gates.data(), sizeof(DevGate) * count, hipMemcpyHostToDevice));
    launch_br(d_gates_, d_ks_, count);
    HIP_CHECK(hipStreamSynchronize(STREAM));
    for (size_t i = 0; i < count; ++i) read_slot(slots[i], out + i * p_.lwe_len());
    for (int s : slots) free_slot(s);
}

void Device::blind_rotate_multi_host(const uint64_t* ks_in, const uint8_t* luts, int n_out, int direct,
                                     uint64_t* out) {
    if (!has_keys()) throw Error(FR_ERR_NO_KEY, "server key not uploaded");
    if (n_out < 1 || n_out > MAX_OUT || direct < 0 || direct > 2 || (direct && n_out != 1))
        throw Error(FR_ERR_INVALID, "bad n_out");
    HIP_CHECK(hipStreamSynchronize(STREAM));  // as blind_rotate_host: queued matches read these buffers
    ensure_batch(1);
    HIP_CHECK(hipMemcpy(d_ks_, ks_in, 8 * (size_t)(p_.n + 1), hipMemcpyHostToDevice));
    DevGate g;
    std::memset(&g, 0, sizeof g);
    g.n_out = n_out;
    g.direct = direct;
    std::vector<int> slots(n_out);
    for (int f = 0; f < n_out; ++f) {
        slots[f] = alloc_slot();
        g.out_slot[f] = slots[f];
        std::memcpy(g.lut[f], luts + 16 * f, 16);
    }
    HIP_CHECK(hipMemcpy(d_gates_, &g, sizeof g, hipMemcpyHostToDevice));
    launch_br(d_gates_, d_ks_, 1);
    HIP_CHECK(hipStreamSynchronize(STREAM));
    for (int f = 0; f < n_out; ++f) read_slot(slots[f], out + (size_t)f * p_.lwe_len());
    for (int sl : slots) free_slot(sl);
}

int lut_w_norm2(const uint8_t* lut) {
    int s = 0;
    for (int m = 1; m < 16; ++m) s += ((int)lut[m] - lut[m - 1]) * ((int)lut[m] - lut[m - 1]);
    s += ((int)lut[0] + lut[15]) * ((int)lut[0] + lut[15]);
    return s;
}

void Device::ring_mul_host(const uint64_t* a, const uint64_t* b, size_t count, uint64_t* out) {
    if (p_.ring != FR_RING_RNS) throw Error(FR_ERR_INVALID, "ring_mul test hook: RNS ring only");
    const int N = p_.N;
    uint64_t *da, *db, *dout;
    HIP_CHECK(hipMalloc(&da, 8 * count * N));
    HIP_CHECK(hipMalloc(&db, 8 * count * N));
    HIP_CHECK(hipMalloc(&dout, 8 * count * N));
    HIP_CHECK(hipMemcpy(da, a, 8 * count * N, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(db, b, 8 * count * N, hipMemcpyHostToDevice));
    // R^2 / N mod p (Montgomery: turns mont(a, b) = ab/R into ab/N)
    uint32_t r2n[2];
    for (int q = 0; q < 2; ++q) {
        const uint64_t pq = rns::prime(q);
        uint64_t inv = 1, b = (uint64_t)N % pq, e = pq - 2;
        while (e) {
            if (e & 1) inv = inv * b % pq;
            b = b * b % pq;
            e >>= 1;
        }
        const uint64_t r2 = q ? rns::R2_1 : rns::R2_0;
        r2n[q] = (uint32_t)(r2 * inv % pq);
    }
    dispatch(p_, e_, [&](auto n_, auto k_, auto e_c) {
        constexpr int NN = decltype(n_)::value, E = decltype(e_c)::value;
        (void)k_;
        const size_t sm = 4 * (4 * (size_t)NttGeo<NN, E>::NP + 2 * (size_t)NN);
        HIP_CHECK(hipFuncSetAttribute((const void*)k_ring_mul<NN, E>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
        k_ring_mul<NN, E><<<(unsigned)count, 4 * (NN / E), sm, STREAM>>>(da, db, d_tw_, r2n[0], r2n[1], dout);
    });
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(STREAM));
    HIP_CHECK(hipMemcpy(out, dout, 8 * count * N, hipMemcpyDeviceToHost));
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
}

void Device::bench_pbs(const std::vector<DevGate>& gates, int iters, double* br_ms, double* total_ms) {
    const size_t n = gates.size();
    ensure_batch(n);
    sync();
    std::memcpy(stage_acquire(), gates.data(), sizeof(DevGate) * n);
    stage_copy(n);
    float br_sum = 0;
    HIP_CHECK(hipEventRecord((hipEvent_t)ev_[3], STREAM));
    for (int it = 0; it < iters; ++it) {
        launch_ks(d_gates_, n, d_ks_);
        HIP_CHECK(hipEventRecord((hipEvent_t)ev_[1], STREAM));
        launch_br(d_gates_, d_ks_, n);
        HIP_CHECK(hipEventRecord((hipEvent_t)ev_[2], STREAM));
        HIP_CHECK(hipEventSynchronize((hipEvent_t)ev_[2]));
        float br = 0;
        HIP_CHECK(hipEventElapsedTime(&br, (hipEvent_t)ev_[1], (hipEvent_t)ev_[2]));
        br_sum += br;
    }
    HIP_CHECK(hipEventRecord((hipEvent_t)ev_[0], STREAM));
    HIP_CHECK(hipEventSynchronize((hipEvent_t)ev_[0]));
    float tot = 0;
    HIP_CHECK(hipEventElapsedTime(&tot, (hipEvent_t)ev_[3], (hipEvent_t)ev_[0]));
    *br_ms = br_sum;
    *total_ms = tot;
}

}  // namespace fr
