// Client key parsing, deterministic server-key generation and client-side
// encryption.  Follows tfhe-rs 0.2 shortint semantics as used by the reference
// (src/regex/ciphertext.rs:32-45, src/regex/engine.rs:248-254): LWE encryption
// under the big (flattened GLWE) key with glwe noise, KSK big->small under the
// LWE noise, GGSW bootstrapping key with one gadget level (g = round(Q/2^23)).
// The GGSW ring is Z_Q[X]/(X^N+1), Q = p0*p1 in RNS form (rns.h).
#include "keys.h"

#include "chacha.h"
#include "rns.h"

#include <atomic>
#include <climits>
#include <cmath>
#include <cstring>
#include <thread>

namespace fr {

// ChaCha20: chacha.h (shared with the device key generator)
uint64_t Rng::u64(uint64_t idx) {
    uint64_t blk = idx >> 3;
    if (!valid_ || blk != blk_) {
        chacha_block(seed_, stream_, blk, w_);
        blk_ = blk;
        valid_ = true;
    }
    int o = (int)(idx & 7) * 2;
    return (uint64_t)w_[o] | ((uint64_t)w_[o + 1] << 32);
}

int64_t Rng::gaussian(uint64_t idx, double sigma, double scale) {
    uint64_t x1 = u64(2 * idx), x2 = u64(2 * idx + 1);
    double u1 = (double)((x1 >> 11) + 1) * 0x1.0p-53;
    double u2 = (double)(x2 >> 11) * 0x1.0p-53;
    double rad = std::sqrt(-2.0 * std::log(u1));
    double z = rad * std::cos(6.283185307179586 * u2);
    double scaled = z * (sigma * scale);
    return (int64_t)std::llround(scaled);
}

using rns::Q;
static inline uint64_t q_add(uint64_t a, uint64_t b) { uint64_t s = a + b; return s >= Q ? s - Q : s; }
static inline uint64_t zq_from_i64(int64_t v) {
    if (v >= 0) return (uint64_t)v % Q;
    uint64_t m = (uint64_t)(-v) % Q;
    return m ? Q - m : 0;
}
static inline uint64_t pow_mod(uint64_t b, uint64_t e, uint64_t p) {
    uint64_t r = 1;
    b %= p;
    while (e) {
        if (e & 1) r = r * b % p;
        b = b * b % p;
        e >>= 1;
    }
    return r;
}

// ---------------------------------------------------------------- key parse
ClientKey parse_client_key(const uint8_t* d, size_t len) {
    size_t off = 0;
    // bounds checks written so that no sum can wrap: a length field of the blob is caller
    // data and may hold any 64-bit value
    auto u = [&](size_t o) -> uint64_t {
        if (o > len || len - o < 8) throw Error(FR_ERR_INVALID, "client key: truncated");
        uint64_t v;
        std::memcpy(&v, d + o, 8);
        return v;
    };
    auto f = [&](size_t o) -> double {
        uint64_t v = u(o);
        double x;
        std::memcpy(&x, &v, 8);
        return x;
    };
    ClientKey ck;
    uint64_t nb = u(off);
    if (nb == 0 || nb > (1u << 20)) throw Error(FR_ERR_INVALID, "client key: bad big key length");
    if (nb > (len - 8) / 8) throw Error(FR_ERR_INVALID, "client key: truncated");
    ck.s_big.resize(nb);
    for (uint64_t i = 0; i < nb; ++i) ck.s_big[i] = u(off + 8 + 8 * i);
    off += 8 + 8 * nb;
    uint64_t ng = u(off);
    if (ng > (len - off - 8) / 8) throw Error(FR_ERR_INVALID, "client key: truncated");
    ck.s_glwe.resize(ng);              // GLWE key data (identical to the big key)
    for (uint64_t i = 0; i < ng; ++i) ck.s_glwe[i] = u(off + 8 + 8 * i);
    off += 8 + 8 * ng;
    ck.glwe_poly_size = u(off);        // polynomial_size
    off += 8;
    uint64_t ns = u(off);
    if (ns == 0 || ns > (1u << 16)) throw Error(FR_ERR_INVALID, "client key: bad small key length");
    if (ns > (len - off - 8) / 8) throw Error(FR_ERR_INVALID, "client key: truncated");
    ck.s_small.resize(ns);
    for (uint64_t i = 0; i < ns; ++i) ck.s_small[i] = u(off + 8 + 8 * i);
    off += 8 + 8 * ns;
    if (u(off) != ns) throw Error(FR_ERR_INVALID, "client key: inconsistent dimensions");
    ck.n = (int)u(off);
    ck.k = (int)u(off + 8);
    ck.N = (int)u(off + 16);
    ck.lwe_sigma = f(off + 24);
    ck.glwe_sigma = f(off + 32);
    ck.pbs_base_log = (int)u(off + 40);
    ck.pbs_level = (int)u(off + 48);
    ck.ks_base_log = (int)u(off + 56);
    ck.ks_level = (int)u(off + 64);
    ck.message_modulus = u(off + 112);
    ck.carry_modulus = u(off + 120);
    ck.num_blocks = u(off + 128);
    for (int i = 0; i < 17; ++i) ck.raw_params[i] = u(off + 8 * (size_t)i);
    if (off + 136 != len) throw Error(FR_ERR_INVALID, "client key: unexpected length");
    for (auto b : ck.s_big)
        if (b > 1) throw Error(FR_ERR_INVALID, "client key: non-binary big key");
    for (auto b : ck.s_small)
        if (b > 1) throw Error(FR_ERR_INVALID, "client key: non-binary small key");
    if ((uint64_t)ck.n != ns || (uint64_t)ck.k * ck.N != nb)
        throw Error(FR_ERR_INVALID, "client key: inconsistent dimensions");
    return ck;
}

std::vector<uint8_t> serialize_client_key(const ClientKey& ck) {
    std::vector<uint8_t> out;
    out.reserve(8 * (ck.s_big.size() + ck.s_glwe.size() + ck.s_small.size() + 21));
    auto put = [&](uint64_t v) {
        uint8_t b[8];
        std::memcpy(b, &v, 8);
        out.insert(out.end(), b, b + 8);
    };
    auto put_vec = [&](const std::vector<uint64_t>& v) {  // bincode Vec<u64>: u64 length, then the words
        put(v.size());
        for (uint64_t x : v) put(x);
    };
    put_vec(ck.s_big);        // lwe_secret_key (the flattened GLWE key)
    put_vec(ck.s_glwe);       // glwe_secret_key: data ...
    put(ck.glwe_poly_size);   // ... and polynomial_size
    put_vec(ck.s_small);      // lwe_secret_key_after_ks
    for (uint64_t w : ck.raw_params) put(w);  // Parameters (16 words) + num_blocks
    return out;
}

ClientKey gen_client_key(const Params& p, uint64_t seed) {
    auto bits = [](double x) {
        uint64_t v;
        std::memcpy(&v, &x, 8);
        return v;
    };
    ClientKey ck;
    const size_t big = (size_t)p.big();
    Rng r(seed, STREAM_CLIENT_KEY);
    // tfhe-rs draws both secret keys as uniform binary vectors; bit 63 of ChaCha word i
    ck.s_big.resize(big);
    for (size_t i = 0; i < big; ++i) ck.s_big[i] = r.u64(i) >> 63;
    ck.s_small.resize((size_t)p.n);
    for (size_t t = 0; t < (size_t)p.n; ++t) ck.s_small[t] = r.u64(big + t) >> 63;
    ck.s_glwe = ck.s_big;
    ck.glwe_poly_size = (uint64_t)p.N;
    ck.n = p.n;
    ck.k = p.k;
    ck.N = p.N;
    ck.pbs_base_log = p.pbs_base_log;
    ck.pbs_level = p.pbs_level;
    ck.ks_base_log = p.ks_base_log;
    ck.ks_level = p.ks_level;
    ck.lwe_sigma = p.lwe_sigma;
    ck.glwe_sigma = p.glwe_sigma;
    ck.message_modulus = 4;
    ck.carry_modulus = 4;
    ck.num_blocks = 4;
    const uint64_t raw[17] = {(uint64_t)p.n, (uint64_t)p.k, (uint64_t)p.N, bits(p.lwe_sigma), bits(p.glwe_sigma),
                              (uint64_t)p.pbs_base_log, (uint64_t)p.pbs_level, (uint64_t)p.ks_base_log,
                              (uint64_t)p.ks_level,
                              1, 23, bits(p.glwe_sigma),  // pfks_level, pfks_base_log, pfks sigma
                              0, 0,                       // cbs_level, cbs_base_log
                              ck.message_modulus, ck.carry_modulus, ck.num_blocks};
    std::memcpy(ck.raw_params, raw, sizeof raw);
    return ck;
}

// ---------------------------------------------------------------- host NTT
static int brv(int x, int bits) {
    int r = 0;
    for (int b = 0; b < bits; ++b)
        if (x >> b & 1) r |= 1 << (bits - 1 - b);
    return r;
}

NttTables::NttTables(int N_) : N(N_) {
    logN = 0;
    while ((1 << logN) < N) ++logN;
    for (int q = 0; q < 2; ++q) {
        const uint64_t p = rns::prime(q);
        const uint64_t psi = pow_mod(rns::GENERATOR, (p - 1) / (2 * (uint64_t)N), p);
        const uint64_t ipsi = pow_mod(psi, p - 2, p);
        zeta[q].resize(N);
        izeta[q].resize(N);
        for (int k = 0; k < N; ++k) {
            zeta[q][k] = (uint32_t)pow_mod(psi, (uint64_t)brv(k, logN), p);
            izeta[q][k] = (uint32_t)pow_mod(ipsi, (uint64_t)brv(k, logN), p);
        }
        n_inv[q] = (uint32_t)pow_mod((uint64_t)N, p - 2, p);
    }
}

void NttTables::forward(int q, uint32_t* a) const {
    const uint64_t p = rns::prime(q);
    for (int s = 0; s < logN; ++s) {
        int L = N >> (s + 1);
        for (int start = 0; start < N; start += 2 * L) {
            uint64_t z = zeta[q][(1 << s) + start / (2 * L)];
            for (int j = start; j < start + L; ++j) {
                uint64_t t = z * a[j + L] % p;
                a[j + L] = (uint32_t)((a[j] + p - t) % p);
                a[j] = (uint32_t)((a[j] + t) % p);
            }
        }
    }
}

void NttTables::inverse(int q, uint32_t* a) const {
    const uint64_t p = rns::prime(q);
    for (int s = logN - 1; s >= 0; --s) {
        int L = N >> (s + 1);
        for (int start = 0; start < N; start += 2 * L) {
            uint64_t z = izeta[q][(1 << s) + start / (2 * L)];
            for (int j = start; j < start + L; ++j) {
                uint64_t u = a[j], v = a[j + L];
                a[j] = (uint32_t)((u + v) % p);
                a[j + L] = (uint32_t)((u + p - v) % p * z % p);
            }
        }
    }
    for (int j = 0; j < N; ++j) a[j] = (uint32_t)((uint64_t)a[j] * n_inv[q] % p);
}

void ring_mul_q(const NttTables& T, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    const int N = T.N;
    std::vector<uint32_t> x[2], y(N);
    for (int q = 0; q < 2; ++q) {
        const uint64_t p = rns::prime(q);
        x[q].resize(N);
        for (int t = 0; t < N; ++t) {
            x[q][t] = (uint32_t)(a[t] % p);
            y[t] = (uint32_t)(b[t] % p);
        }
        T.forward(q, x[q].data());
        T.forward(q, y.data());
        for (int t = 0; t < N; ++t) x[q][t] = (uint32_t)((uint64_t)x[q][t] * y[t] % p);
        T.inverse(q, x[q].data());
    }
    for (int t = 0; t < N; ++t) out[t] = rns::crt(x[0][t], x[1][t]);
}

// ---------------------------------------------------------------- keygen
template <class F>
static void parallel_for(int n, F&& fn) {
    unsigned hw = std::thread::hardware_concurrency();
    int T = (int)(hw ? (hw > 16 ? 16 : hw) : 4);
    if (T > n) T = n > 0 ? n : 1;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (int i = t; i < n; i += T) fn(i);
        });
    for (auto& x : th) x.join();
}

void gen_ksk(const Params& p, const ClientKey& ck, uint64_t seed, std::vector<uint64_t>& ksk) {
    const int big = p.big(), n = p.n, L = p.ks_level, B = p.ks_base_log;
    ksk.assign((size_t)big * L * (n + 1), 0);
    parallel_for(big, [&](int i) {
        Rng rm(seed, STREAM_KSK_MASK), rn(seed, STREAM_KSK_NOISE);
        for (int j = 0; j < L; ++j) {
            uint64_t row = (uint64_t)i * L + j;
            uint64_t* o = ksk.data() + row * (n + 1);
            uint64_t body = 0;
            for (int t = 0; t < n; ++t) {
                o[t] = rm.u64(row * n + t);
                body += o[t] * ck.s_small[t];
            }
            body += ck.s_big[i] << (64 - B * (j + 1));
            body += (uint64_t)rn.gaussian(row, p.lwe_sigma);
            o[n] = body;
        }
    });
}

// message bit of GGSW number w (see Params::bsk_unroll)
static uint64_t ggsw_msg(const Params& p, const ClientKey& ck, size_t w) {
    if (p.bsk_unroll() == 1) return ck.s_small[w];
    const size_t t = w / 3, g = w % 3, i = 2 * t, j = 2 * t + 1;
    const uint64_t si = ck.s_small[i], sj = j < (size_t)p.n ? ck.s_small[j] : 0;
    return g == 0 ? (si & sj) : g == 1 ? (si & (1 - sj)) : ((1 - si) & sj);
}

// Torus BSK (FR_RING_FFT): row r of GGSW w is a GLWE encryption of zero on the
// 2^64 torus (mask uniform u64, body = sum_j A_j S_j + e, e ~ sigma_glwe 2^64),
// plus m_w * 2^(64 - B) (the one-level gadget, B = pbs_base_log) on coefficient
// 0 of component r.  A_j S_j (binary S) is summed exactly as rotations of A.
static void gen_bsk_torus(const Params& p, const ClientKey& ck, uint64_t seed, std::vector<uint64_t>& bsk) {
    const int k = p.k, N = p.N;
    const size_t kp1 = (size_t)k + 1, nw = p.bsk_ggsw();
    const uint64_t gadget = 1ULL << (64 - p.pbs_base_log);
    bsk.assign(p.bsk_len(), 0);
    parallel_for((int)nw, [&](int i) {
        Rng rm(seed, STREAM_BSK_MASK), rn(seed, STREAM_BSK_NOISE);
        const uint64_t msg = ggsw_msg(p, ck, (size_t)i);
        for (size_t r = 0; r < kp1; ++r) {
            uint64_t* row = bsk.data() + ((size_t)i * kp1 + r) * kp1 * N;
            uint64_t* Bp = row + (size_t)k * N;
            for (int j = 0; j < k; ++j) {
                uint64_t* A = row + (size_t)j * N;
                const uint64_t base = (((uint64_t)i * kp1 + r) * k + j) * N;
                for (int t = 0; t < N; ++t) A[t] = rm.u64(base + t);
                const uint64_t* S = ck.s_big.data() + (size_t)j * N;
                for (int u = 0; u < N; ++u) {
                    if (!S[u]) continue;
                    // X^u A: coefficient t + u gets A[t] (t + u < N), -A[t] past the wrap
                    for (int t = 0; t < N - u; ++t) Bp[t + u] += A[t];
                    for (int t = N - u; t < N; ++t) Bp[t + u - N] -= A[t];
                }
            }
            const uint64_t nb = ((uint64_t)i * kp1 + r) * N;
            for (int t = 0; t < N; ++t) Bp[t] += (uint64_t)rn.gaussian(nb + t, p.glwe_sigma);
            if (msg) row[r * N] += gadget;
        }
    });
}

// noise terms of the device key generator (keygen.hip): the same draws as
// gen_ksk / gen_bsk_torus above (Box-Muller stays on the host, where libm is
// the reference for the bits)
void gen_ksk_noise(const Params& p, uint64_t seed, std::vector<int64_t>& e) {
    const size_t rows = (size_t)p.big() * p.ks_level;
    e.resize(rows);
    Rng rn(seed, STREAM_KSK_NOISE);
    for (size_t row = 0; row < rows; ++row) e[row] = rn.gaussian(row, p.lwe_sigma);
}
void gen_bsk_noise_torus(const Params& p, uint64_t seed, std::vector<int32_t>& e) {
    const size_t polys = p.bsk_ggsw() * (size_t)(p.k + 1), N = (size_t)p.N;
    e.resize(polys * N);
    std::atomic<bool> ok{true};
    parallel_for((int)polys, [&](int q) {
        Rng rn(seed, STREAM_BSK_NOISE);
        for (size_t t = 0; t < N; ++t) {
            const int64_t v = rn.gaussian((uint64_t)q * N + t, p.glwe_sigma);
            if (v < INT32_MIN || v > INT32_MAX) ok = false;
            e[(size_t)q * N + t] = (int32_t)v;
        }
    });
    if (!ok) throw Error(FR_ERR_INVALID, "GLWE noise outside int32 (sigma too large for the device key generator)");
}
void enc_noise(const Params& p, uint64_t seed, uint64_t first_block, size_t count, std::vector<int64_t>& e) {
    e.resize(count);
    Rng rn(seed, STREAM_ENC_NOISE);
    for (size_t q = 0; q < count; ++q) e[q] = rn.gaussian(first_block + q, p.glwe_sigma);
}
std::vector<uint8_t> ggsw_messages(const Params& p, const ClientKey& ck) {
    std::vector<uint8_t> m(p.bsk_ggsw());
    for (size_t w = 0; w < m.size(); ++w) m[w] = (uint8_t)ggsw_msg(p, ck, w);
    return m;
}

void gen_bsk(const Params& p, const ClientKey& ck, uint64_t seed, std::vector<uint64_t>& bsk) {
    if (p.ring == FR_RING_FFT) {
        gen_bsk_torus(p, ck, seed, bsk);
        return;
    }
    const int k = p.k, N = p.N;
    const size_t kp1 = (size_t)k + 1, nw = p.bsk_ggsw();
    bsk.assign(p.bsk_len(), 0);
    NttTables T(N);
    // NTT of the key polynomials S_j, per prime
    std::vector<uint32_t> S[2];
    for (int q = 0; q < 2; ++q) {
        S[q].resize((size_t)k * N);
        for (int j = 0; j < k; ++j) {
            for (int t = 0; t < N; ++t) S[q][(size_t)j * N + t] = (uint32_t)ck.s_big[(size_t)j * N + t];
            T.forward(q, S[q].data() + (size_t)j * N);
        }
    }
    parallel_for((int)nw, [&](int i) {
        Rng rm(seed, STREAM_BSK_MASK), rn(seed, STREAM_BSK_NOISE);
        std::vector<uint32_t> tmp(N), acc[2] = {std::vector<uint32_t>(N), std::vector<uint32_t>(N)};
        const uint64_t msg = ggsw_msg(p, ck, (size_t)i);
        for (size_t r = 0; r < kp1; ++r) {
            uint64_t* row = bsk.data() + ((size_t)i * kp1 + r) * kp1 * N;
            std::fill(acc[0].begin(), acc[0].end(), 0);
            std::fill(acc[1].begin(), acc[1].end(), 0);
            for (int j = 0; j < k; ++j) {
                uint64_t* A = row + (size_t)j * N;
                uint64_t base = (((uint64_t)i * kp1 + r) * k + j) * N;
                // uniform mask in [0, Q): floor(x * Q / 2^64)
                for (int t = 0; t < N; ++t) A[t] = (uint64_t)(((unsigned __int128)rm.u64(base + t) * Q) >> 64);
                for (int q = 0; q < 2; ++q) {
                    const uint64_t pq = rns::prime(q);
                    for (int t = 0; t < N; ++t) tmp[t] = (uint32_t)(A[t] % pq);
                    T.forward(q, tmp.data());
                    const uint32_t* Sj = S[q].data() + (size_t)j * N;
                    for (int t = 0; t < N; ++t) acc[q][t] = (uint32_t)((acc[q][t] + (uint64_t)tmp[t] * Sj[t]) % pq);
                }
            }
            T.inverse(0, acc[0].data());
            T.inverse(1, acc[1].data());
            uint64_t* Bp = row + (size_t)k * N;
            uint64_t nb = ((uint64_t)i * kp1 + r) * N;
            for (int t = 0; t < N; ++t)
                Bp[t] = q_add(rns::crt(acc[0][t], acc[1][t]), zq_from_i64(rn.gaussian(nb + t, p.glwe_sigma, (double)Q)));
            if (msg) row[r * N] = q_add(row[r * N], rns::G);
        }
    });
}

// ---------------------------------------------------------------- client
void encrypt_blocks(const Params& p, const ClientKey& ck, const uint8_t* msgs, size_t count, uint64_t seed,
                    uint64_t first_block, uint64_t* out) {
    const int big = p.big();
    Rng rm(seed, STREAM_ENC_MASK), rn(seed, STREAM_ENC_NOISE);
    for (size_t q = 0; q < count; ++q) {
        uint64_t* o = out + q * (big + 1);
        uint64_t qb = first_block + q, body = 0;
        for (int t = 0; t < big; ++t) {
            o[t] = rm.u64(qb * big + t);
            body += o[t] * ck.s_big[t];
        }
        body += (uint64_t)msgs[q] << DELTA_LOG;
        body += (uint64_t)rn.gaussian(qb, p.glwe_sigma);
        o[big] = body;
    }
}

uint64_t lwe_phase(const Params& p, const ClientKey& ck, const uint64_t* lwe) {
    const int big = p.big();
    uint64_t acc = lwe[big];
    for (int t = 0; t < big; ++t) acc -= lwe[t] * ck.s_big[t];
    return acc;
}

uint32_t decode16(uint64_t phase) {
    const uint64_t delta = 1ULL << DELTA_LOG;
    uint64_t rounding = (phase & (delta >> 1)) << 1;
    return (uint32_t)(((phase + rounding) / delta) % 16);
}

}  // namespace fr
