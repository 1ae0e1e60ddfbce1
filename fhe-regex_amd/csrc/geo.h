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
// dword address mod 32 (MI355X_MICROARCH.md §LDS).  Generally: groups of 2^GB
// lanes, 2^GB bank units (GB = 5 for b32; the b128 accesses of the f64 FFT,
// GB = 3, follow gfx950's own read and write groups: make_b128_map below).  In every phase
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
// Layout p sends lane bit b to index bit geo_lane_bit(.., p, b); phase p's E elements
// are the index bits [lo(p), lo(p) + e).  Layout family V:
//  V = 0: lane bits keep their order around the element bits (b < lo(p): b, else b + e).
//  V = 1 (M = 1024, E = 4, 256 lanes: the f64 FFT of k = 1): layouts 3 and 4 put lane
//    bits 0..3 on index bits 4, 5, 7, 6 (bit 6 last: it is lane bit 4 of layout 2, whose
//    b128 reads want it off the write groups' lane bits 0..2 of layout 3) and lane bits
//    4, 5 on the other phase's element bits
//    (layout 3: 0, 1; layout 4: 2, 3), so that the exchange 3 <-> 4, like 1 <-> 2,
//    swaps element bits with lane bits 4 and 5 (v_permlane16/32_swap, no LDS); the
//    other layouts are V = 0's.
constexpr int geo_lane_bit(int LOG, int e, int p, int b, int V = 0) {
    if (V == 1 && p >= 3) {
        if (b < 4) return b < 2 ? 4 + b : 9 - b;
        if (b < 6) return (p == 3 ? 0 : 2) + (b - 4);
        return b + 2;
    }
    return b < geo_lo(LOG, e, p) ? b : b + e;
}
// index of element 0 of lane tl in layout p (host and compile-time use)
constexpr int geo_base(int LOG, int e, int p, int tl, int V = 0) {
    int idx = 0;
    for (int b = 0; (tl >> b) != 0; ++b)
        if ((tl >> b) & 1) idx |= 1 << geo_lane_bit(LOG, e, p, b, V);
    return idx;
}
// the layout family of the f64 FFT kernels (fft_br.hip, keygen.hip, the key upload)
constexpr int fft_layout_variant(int LOG, int e) { return LOG == 10 && e == 2 ? 1 : 0; }
constexpr unsigned geo_group(int LOG, int e, int p, int GB, int V = 0) {
    unsigned g = 0;
    for (int b = 0; b < GB; ++b) g |= 1u << geo_lane_bit(LOG, e, p, b, V);
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
// gfx950 b128 accesses (one complex f64, fft_br.hip; MI355X_MICROARCH.md §LDS):
//  * ds_write_b128 is served in 8 groups of 8 contiguous lanes, bank quad (a/16) mod 8;
//  * ds_read_b128 in 4 groups of 16 lanes -- {0-3,12-15,20-27}, {4-11,16-19,28-31} and
//    the same +32, i.e. (lane bit 5, parity of lane bits 2..4) -- bank quad (a/16) mod 16.
// An exchange map (both directions: forward writes layout x and reads x+1, the inverse
// writes x+1 and reads x; map NPH-2 also serves the MAC's last-layout accesses) is
// conflict-free for both when, with v(k) the 2-adic valuation of the weight of index
// bit k:
//  * the index bits of lane bits 0..2 in a written layout take v = {0, 1, 2};
//  * the index bits of lane bits 0..3 in a read layout take v = {0, 1, 2, 3} and that
//    of lane bit 4 takes v >= 4 (then lane bit 4, which the group couples to bits 2
//    and 3, adds a multiple of 16).
// make_b128_map solves these valuation constraints by backtracking and then picks the
// smallest injective additive weights greedily (low valuations first), which keeps the
// row span near 2^H.
constexpr int b128_rgroup(int lane) { return ((lane >> 5) << 1) | (((lane >> 2) ^ (lane >> 3) ^ (lane >> 4)) & 1); }
struct B128Req {
    int nset = 0;
    int set[8][5] = {};  // index bits that need distinct valuations {0..size-1}
    int size[8] = {};
    int ge4[4] = {};     // index bits that need valuation >= 4
    int nge4 = 0;
};
// map x serves the exchange x <-> x+1; with V = 1 the exchange (nph-2) <-> (nph-1) is a
// register exchange and map nph-2 serves only the MAC's last-layout accesses
constexpr bool b128_mac_only(int x, int nph, int V) { return V == 1 && x == nph - 2; }
// V = 1, exchange 2 <-> 3: index bit 6 is lane bit 4 of layout 2 and one of lane bits 0..3
// of layout 3 (index bit 0 the other way round), so the reads of one of the two layouts
// cannot be conflict-free; layout 3's reads (the forward exchange) take 2-way conflicts
constexpr int b128_relaxed_read(int x, int V) { return V == 1 && x == 2 ? 3 : -1; }
constexpr B128Req b128_requirements(int LOG, int e, int x, int nph, int V = 0) {
    B128Req q{};
    const int xt = x + 1 < nph ? x + 1 : x;
    const int xf = b128_mac_only(x, nph, V) ? xt : x;
    const int dirs[2][2] = {{xf, xt}, {xt, xf}};  // (written layout, read layout)
    for (int d = 0; d < 2; ++d) {
        const int W = dirs[d][0], R = dirs[d][1];
        q.size[q.nset] = 3;
        for (int b = 0; b < 3; ++b) q.set[q.nset][b] = geo_lane_bit(LOG, e, W, b, V);
        ++q.nset;
        if (R == b128_relaxed_read(x, V)) continue;
        q.size[q.nset] = 4;
        for (int b = 0; b < 4; ++b) q.set[q.nset][b] = geo_lane_bit(LOG, e, R, b, V);
        ++q.nset;
        q.ge4[q.nge4++] = geo_lane_bit(LOG, e, R, 4, V);
    }
    return q;
}
// partial check of valuations val[0..k] (4 = ">= 4", -1 = unassigned)
constexpr bool b128_partial_ok(const B128Req& q, const int* val) {
    for (int i = 0; i < q.nge4; ++i)
        if (val[q.ge4[i]] >= 0 && val[q.ge4[i]] != 4) return false;
    for (int s = 0; s < q.nset; ++s) {
        bool used[5] = {};
        for (int i = 0; i < q.size[s]; ++i) {
            const int v = val[q.set[s][i]];
            if (v < 0) continue;
            if (v >= q.size[s] || used[v]) return false;
            used[v] = true;
        }
    }
    return true;
}
constexpr bool b128_solve(const B128Req& q, int* val, int k, int H) {
    if (k == H) return true;
    const int order[5] = {4, 0, 1, 2, 3};
    for (int t = 0; t < 5; ++t) {
        val[k] = order[t];
        if (b128_partial_ok(q, val) && b128_solve(q, val, k + 1, H)) return true;
    }
    val[k] = -1;
    return false;
}
constexpr int val2(int w) {
    int v = 0;
    while (!(w & 1) && v < 4) {
        w >>= 1;
        ++v;
    }
    return v;
}
constexpr LdsMap make_b128_map(int LOG, int e, int H, int x, int nph, int V = 0) {
    LdsMap m{};
    const B128Req q = b128_requirements(LOG, e, x, nph, V);
    int val[16] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
    if (!b128_solve(q, val, 0, H)) {
        m.span = -1;  // caught by the conflict check
        return m;
    }
    // greedy order: the first bit of each valuation 0..3, then the v >= 4 bits, then the rest
    int order[16] = {}, no = 0;
    bool taken[16] = {};
    for (int v = 0; v < 4; ++v)
        for (int k = 0; k < H; ++k)
            if (!taken[k] && val[k] == v) {
                order[no++] = k;
                taken[k] = true;
                break;
            }
    for (int k = 0; k < H; ++k)
        if (!taken[k] && val[k] == 4) order[no++] = k, taken[k] = true;
    for (int k = 0; k < H; ++k)
        if (!taken[k]) order[no++] = k, taken[k] = true;
    bool reach[2048] = {};
    reach[0] = true;
    int top = 0;
    for (int i = 0; i < no; ++i) {
        const int k = order[i];
        for (int w = 1;; ++w) {
            if (val2(w) != val[k]) continue;
            if (top + w >= 2048) {
                m.span = -1;
                return m;
            }
            bool clash = false;
            for (int s = 0; s <= top && !clash; ++s) clash = reach[s] && reach[s + w];
            if (clash) continue;
            for (int s = top; s >= 0; --s)
                if (reach[s]) reach[s + w] = true;
            top += w;
            m.w[k] = w;
            break;
        }
    }
    m.span = (top + 1 + 15) / 16 * 16;
    return m;
}
struct LdsMaps {
    LdsMap m[12];
    int ch;
};
constexpr LdsMaps make_lds_maps(int LOG, int e, int H, int nph, int GB, int V = 0) {
    LdsMaps r{};
    r.ch = 1 << GB;
    for (int x = 0; x < (nph > 1 ? nph - 1 : 1); ++x) {
        r.m[x] = GB == 3 ? make_b128_map(LOG, e, H, x, nph, V) : make_lds_map(LOG, e, H, x, nph, GB);
        if (r.m[x].span > r.ch) r.ch = r.m[x].span;
    }
    return r;
}

// N-point negacyclic NTT spread over T = N/E lanes holding E coefficients
// each.  The LOG = log2 N stages run as NPH register-resident phases of e =
// log2 E stages; phase p's lane owns the E elements that differ in index bits
// [lo(p), lo(p)+e), and two consecutive phases are joined by one LDS
// exchange.  Forward stage s pairs bit LOG-1-s with zeta[(1<<s) + (j >> (LOG-s))].
template <int N, int E, int GB = 5, int V = 0>
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
    static constexpr LdsMaps MAPS = make_lds_maps(LOG, e, H, NPH, GB, V);
    static_assert(V == 0 || (LOG == 10 && e == 2 && T == 256), "layout family V = 1: M = 1024, E = 4");
    static constexpr int lane_bit(int p, int b) { return geo_lane_bit(LOG, e, p, b, V); }
    static constexpr int CH = MAPS.ch;
    static constexpr int NP = CH << WB;  // LDS row (elements)
    static constexpr int XL = NPH >= 2 ? NPH - 2 : 0;
    // the wave bits of layout p are its top index bits [H, LOG)
    static constexpr bool wave_top(int p) { return WB == 0 || lo(p) <= 6; }
    static_assert(V == 0 || (lane_bit(3, 6) == 8 && lane_bit(4, 7) == 9), "V = 1 keeps the wave bits on top");
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
            const int b = at<X>(geo_base(LOG, e, p, l, V)) & ((1 << GB) - 1);
            if (seen[b]) return false;
            seen[b] = true;
        }
        return true;
    }
    // gfx950 b128 conflict check of exchange map X (see make_b128_map): the writes of
    // the written layout hit 8 distinct bank quads per 8-lane group, the reads of the
    // read layout 16 distinct quads per read group, in both directions
    // (max_way: the largest number of a group's lanes allowed on one bank quad)
    template <int X>
    static constexpr bool b128_layout_ok(int p, bool write, int max_way = 1) {
        for (int g = 0; g < (write ? 8 : 4); ++g) {
            int seen[16] = {};
            for (int l = 0; l < 64; ++l) {
                if ((write ? l >> 3 : b128_rgroup(l)) != g) continue;
                const int b = at<X>(geo_base(LOG, e, p, l, V)) & (write ? 7 : 15);
                if (++seen[b] > max_way) return false;
            }
        }
        return true;
    }
    // map X sends the N indices of a row to distinct addresses inside the row (NP slots)
    template <int X>
    static constexpr bool map_injective() {
        bool seen[NP] = {};
        for (int i = 0; i < N; ++i) {
            const int a = at<X>(i);
            if (a < 0 || a >= NP || seen[a]) return false;
            seen[a] = true;
        }
        return true;
    }
    template <int X>
    static constexpr bool b128_exchange_ok() {
        const int xt = X + 1 < NPH ? X + 1 : X;
        const int xf = b128_mac_only(X, NPH, V) ? xt : X;
        const int rw = b128_relaxed_read(X, V);
        return MAPS.m[X].span > 0 && map_injective<X>() && b128_layout_ok<X>(xf, true) &&
               b128_layout_ok<X>(xt, false, xt == rw ? 2 : 1) && b128_layout_ok<X>(xt, true) &&
               b128_layout_ok<X>(xf, false, xf == rw ? 2 : 1);
    }
    // element m of lane tl in phase p: idx = base(tl) | moff(m), disjoint bits,
    // so at(idx) = at(base) + at(moff): every address is one per-lane register
    // plus a compile-time immediate.
    template <int p>
    __device__ static __forceinline__ int base(int tl) {
        if constexpr (V == 1 && p >= 3) {  // lane bits 0..3 -> index 4, 5, 7, 6
            return ((tl & 3) << 4) | ((tl & 4) << 5) | ((tl & 8) << 3) | (((tl >> 4) & 3) << (p == 3 ? 0 : 2)) |
                   ((tl >> 6) << 8);
        } else {
            constexpr int L = lo(p);
            return ((tl >> L) << (L + e)) | (tl & ((1 << L) - 1));
        }
    }
    template <int p>
    static constexpr int moff(int m) { return m << lo(p); }
    template <int p>
    __device__ static __forceinline__ int idx(int tl, int m) { return base<p>(tl) + moff<p>(m); }
};


}  // namespace fr
