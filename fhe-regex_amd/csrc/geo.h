// Lane geometry of the register-phase NTT/FFT kernels and their bank-conflict-
// free LDS exchange maps (shared by device.hip: RNS NTT, and fft.hip: f64 FFT).
#pragma once
#include <hip/hip_runtime.h>

namespace fr {

// ------------------------------------------------------------------ geometry
constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x / 2); }

// LDS address maps of an exchange row (bank-conflict-free exchanges).
//
// A b32 LDS access of a wave is served in two 32-lane groups with bank =
// dword address mod 32 (MI355X_MICROARCH.md §LDS); a b128 access (one complex
// f64, fft.hip) in eight 8-lane groups of 16-B bank quads.  Generally: groups
// of 2^GB lanes, 2^GB bank units (GB = 5 for b32, 3 for b128).  In every phase
// layout the lanes of a group vary GB index bits (the "group bits" of the layout),
// so an exchange between phases p and p+1 is conflict-free iff the address map
// sends each of the two group-bit sets to 2^GB distinct bank units.  An additive map
// addr(i) = sum_k w_k * bit_k(i) does that iff, within each group, the 2-adic
// valuations of the w_k mod 2^GB are exactly {0..GB-1}; no single additive map can
// serve all four layouts of N = 2048, E = 8 (the constraints of P0/P2/P3
// contradict), so each exchange (p, p+1) gets its own map.  Additive maps keep
// every address one per-lane register plus a compile-time immediate.
//
// Construction: shared group bits and pairs (i-th private bit of each group)
// take valuations 0, 1, ... in ascending bit order; weights are then the
// smallest superincreasing values with those valuations (injective).  The wave
// bits of a row (top index bits in layouts p >= 1, see wave_top) get a weight
// CH * 2^j common to all maps, so in those layouts a wave's slots form the
// same address chunk under every map, which is what keeps the barrier plan
// below valid across map changes.
struct LdsMap {
    int w[16];
    int span;
};
constexpr int geo_lo(int LOG, int e, int p) { return LOG - (p + 1) * e > 0 ? LOG - (p + 1) * e : 0; }
constexpr int geo_lane_bit(int LOG, int e, int p, int b) { return b < geo_lo(LOG, e, p) ? b : b + e; }
constexpr unsigned geo_group(int LOG, int e, int p, int GB) {
    unsigned g = 0;
    for (int b = 0; b < GB; ++b) g |= 1u << geo_lane_bit(LOG, e, p, b);
    return g;
}
constexpr LdsMap make_lds_map(int LOG, int e, int H, int x, int nph, int GB) {
    LdsMap m{};
    const unsigned F = geo_group(LOG, e, x, GB), Tg = geo_group(LOG, e, x + 1 < nph ? x + 1 : x, GB), S = F & Tg;
    int color[16] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
    int pf[5] = {0, 0, 0, 0, 0}, pt[5] = {0, 0, 0, 0, 0};
    int nf = 0, nt = 0;
    for (int k = 0; k < LOG; ++k) {
        if (((F >> k) & 1) && !((S >> k) & 1)) pf[nf++] = k;
        if (((Tg >> k) & 1) && !((S >> k) & 1)) pt[nt++] = k;
    }
    int next = 0;
    for (int k = 0; k < LOG; ++k) {
        if (color[k] >= 0) continue;
        if ((S >> k) & 1) {
            color[k] = next++;
            continue;
        }
        for (int i = 0; i < nf; ++i)
            if (pf[i] == k || pt[i] == k) {
                color[pf[i]] = color[pt[i]] = next++;
                break;
            }
    }
    int sum = 0;
    for (int k = 0; k < H; ++k) {
        int w = sum + 1;
        if (color[k] >= 0)
            while (w % (2 << color[k]) != (1 << color[k])) ++w;
        m.w[k] = w;
        sum += w;
    }
    m.span = (sum + (1 << GB)) / (1 << GB) * (1 << GB);
    return m;
}
struct LdsMaps {
    LdsMap m[8];
    int ch;
};
constexpr LdsMaps make_lds_maps(int LOG, int e, int H, int nph, int GB) {
    LdsMaps r{};
    r.ch = 1 << GB;
    for (int x = 0; x < (nph > 1 ? nph - 1 : 1); ++x) {
        r.m[x] = make_lds_map(LOG, e, H, x, nph, GB);
        if (r.m[x].span > r.ch) r.ch = r.m[x].span;
    }
    return r;
}

// N-point negacyclic NTT spread over T = N/E lanes holding E coefficients
// each.  The LOG = log2 N stages run as NPH register-resident phases of e =
// log2 E stages; phase p's lane owns the E elements that differ in index bits
// [lo(p), lo(p)+e), and two consecutive phases are joined by one LDS
// exchange.  Forward stage s pairs bit LOG-1-s with zeta[(1<<s) + (j >> (LOG-s))].
template <int N, int E, int GB = 5>
struct NttGeo {
    static constexpr int LOG = ilog2c(N);
    static constexpr int e = ilog2c(E);
    static constexpr int T = N / E;
    static constexpr int NPH = (LOG + e - 1) / e;
    static_assert((1 << LOG) == N && (1 << e) == E, "powers of two");
    static_assert(T % 64 == 0, "a (polynomial, prime) pair must own whole waves");
    static constexpr int lo(int p) { return geo_lo(LOG, e, p); }
    static constexpr int s_begin(int p) { return p * e; }
    static constexpr int s_end(int p) { return (p + 1) * e < LOG ? (p + 1) * e : LOG; }
    // LDS address maps (above): map X serves the exchange between phases X and
    // X+1; map 0 also serves natural-order (phase-0) accesses, map XL the
    // last-phase (bit-reversed slot) accesses of the MAC.
    static constexpr int WB = ilog2c(T / 64);  // wave bits of a row
    static constexpr int H = LOG - WB;
    static constexpr LdsMaps MAPS = make_lds_maps(LOG, e, H, NPH, GB);
    static constexpr int CH = MAPS.ch;
    static constexpr int NP = CH << WB;  // LDS row (elements)
    static constexpr int XL = NPH >= 2 ? NPH - 2 : 0;
    // the wave bits of layout p are its top index bits [H, LOG)
    static constexpr bool wave_top(int p) { return WB == 0 || lo(p) <= 6; }
    template <int X>
    static constexpr int wt(int k) {
        return k < H ? MAPS.m[X].w[k] : CH << (k - H);
    }
    // address of index i under map X (constant-folds for constant i; at run
    // time only the bits whose weight differs from 2^k cost an operation)
    template <int X>
    __host__ __device__ static constexpr int at(int i) {
        int a = i;
#pragma unroll
        for (int k = 0; k < LOG; ++k)
            if (wt<X>(k) != (1 << k)) a += ((i >> k) & 1) * (wt<X>(k) - (1 << k));
        return a;
    }
    // conflict check: the 2^GB lanes of a group in layout p under map X hit distinct bank units
    template <int X>
    static constexpr bool banks_distinct(int p) {
        bool seen[32] = {};
        for (int l = 0; l < (1 << GB); ++l) {
            const int b = at<X>(((l >> lo(p)) << (lo(p) + e)) | (l & ((1 << lo(p)) - 1))) & ((1 << GB) - 1);
            if (seen[b]) return false;
            seen[b] = true;
        }
        return true;
    }
    // element m of lane tl in phase p: idx = base(tl) | moff(m), disjoint bits,
    // so at(idx) = at(base) + at(moff): every address is one per-lane register
    // plus a compile-time immediate.
    template <int p>
    __device__ static __forceinline__ int base(int tl) {
        constexpr int L = lo(p);
        return ((tl >> L) << (L + e)) | (tl & ((1 << L) - 1));
    }
    template <int p>
    static constexpr int moff(int m) { return m << lo(p); }
    template <int p>
    __device__ static __forceinline__ int idx(int tl, int m) { return base<p>(tl) + moff<p>(m); }
};


}  // namespace fr
