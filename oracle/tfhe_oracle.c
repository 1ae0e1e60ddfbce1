/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library,
 * and only as the checker / CPU baseline, never as the thing measured.
 *
 * CPU restatement of the gate-bootstrap path under the reference's regex
 * engine.  The reference delegates all homomorphic arithmetic to the git
 * dependency tfhe-rs 0.2.0 (zama-ai/tfhe-rs @ 13ad7d5, reference Cargo.lock:
 * 602-615; features integer+shortint, Cargo.toml:8), which is ABSENT from
 * /root/reference and cannot be fetched.  This file restates tfhe-rs 0.2's
 * published shortint PBS algorithm (KS-first order: keyswitch -> modulus
 * switch -> blind rotation -> sample extract) at the parameters decoded from
 * the reference fixture test_data/client_key (PARAM_MESSAGE_2_CARRY_2:
 * n=742, k=1, N=2048, PBS 2^23 x 1, KS 2^3 x 5, Delta = 2^59), with one
 * documented deviation shared with the GPU product: the GLWE/GGSW ring is
 * Z_p[X]/(X^N+1) with p = 2^64 - 2^32 + 1 (exact integer NTT) instead of
 * tfhe-rs's torus 2^64 with an f64 FFT; sample-extracted LWEs are mapped back
 * to the 2^64 torus by x -> round(x * 2^64 / p) so every ciphertext that
 * crosses the boundary decrypts with the reference's client key and the
 * tfhe-rs decoding rule (shortint decrypt_message_and_carry).
 *
 * Call sites in the reference this path replaces: src/regex/execution.rs:76,
 * 93,110,143,173,190 (smart_eq/gt/le/bitand/bitor/bitxor), trivial constants
 * src/regex/ciphertext.rs:8-30, keygen src/regex/ciphertext.rs:42-45 and
 * engine.rs:252 (ServerKey::new).
 *
 * Parity pins: the fixture client key (decoding verified in tests), the 25
 * decrypted-result cases of src/regex/engine.rs:256-280, and bit-identity with
 * the GPU path (same keys, same inputs).  The ring product here is a textbook
 * twisted cyclic NTT, written independently of the GPU's merged-psi NTT; both
 * are exact in Z_p so the products agree bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

#define GL_P 0xFFFFFFFF00000001ULL

/* ---------------------------------------------------------------- params */
typedef struct {
    int32_t k;            /* GLWE dimension */
    int32_t N;            /* polynomial size */
    int32_t n;            /* small LWE dimension */
    int32_t ks_base_log;  /* 3 */
    int32_t ks_level;     /* 5 */
    int32_t pbs_base_log; /* 23 */
    int32_t pbs_level;    /* 1 */
    int32_t _pad;
    double lwe_sigma;     /* KSK noise (std dev as a fraction of the torus) */
    double glwe_sigma;    /* BSK / fresh-encryption noise */
} or_params;

/* ----------------------------------------------------------- Goldilocks */
static inline uint64_t gl_reduce128(u128 x) {
    /* x = lo + hl*2^64 + hh*2^96 ; 2^64 = 2^32-1, 2^96 = -1 (mod p) */
    uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    uint64_t hh = hi >> 32, hl = hi & 0xFFFFFFFFULL;
    uint64_t t = lo - hh;
    if (lo < hh) t -= 0xFFFFFFFFULL;            /* borrow: + p */
    uint64_t u = hl * 0xFFFFFFFFULL;
    uint64_t r = t + u;
    if (r < t) r += 0xFFFFFFFFULL;              /* carry: + 2^64 = 2^32-1 */
    return r >= GL_P ? r - GL_P : r;
}
static inline uint64_t gl_add(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    if (s < a) s += 0xFFFFFFFFULL;
    return s >= GL_P ? s - GL_P : s;
}
static inline uint64_t gl_sub(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (GL_P - b); }
static inline uint64_t gl_mul(uint64_t a, uint64_t b) { return gl_reduce128((u128)a * b); }
static uint64_t gl_pow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    while (e) { if (e & 1) r = gl_mul(r, b); b = gl_mul(b, b); e >>= 1; }
    return r;
}
static inline uint64_t gl_from_i64(int64_t v) { return v >= 0 ? (uint64_t)v % GL_P : GL_P - ((uint64_t)(-v) % GL_P); }

uint64_t or_gl_mul(uint64_t a, uint64_t b) { return gl_mul(a, b); }

/* ------------------------------------------------------------- ChaCha20 */
#define ROTL32(a, b) (((a) << (b)) | ((a) >> (32 - (b))))
#define QR(a, b, c, d) \
    a += b; d ^= a; d = ROTL32(d, 16); c += d; b ^= c; b = ROTL32(b, 12); \
    a += b; d ^= a; d = ROTL32(d, 8);  c += d; b ^= c; b = ROTL32(b, 7);

static void chacha20_block(uint64_t seed, uint64_t stream, uint64_t counter, uint32_t out[16]) {
    uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                       (uint32_t)seed, (uint32_t)(seed >> 32), 0x243F6A88u, 0x85A308D3u,
                       0x13198A2Eu, 0x03707344u, 0xA4093822u, 0x299F31D0u,
                       (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
    uint32_t x[16];
    memcpy(x, in, sizeof x);
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

/* u64 number `idx` of stream (seed, stream): block idx/8, words 2*(idx%8), +1 */
typedef struct { uint64_t seed, stream, blk; uint32_t w[16]; int valid; } rng_t;
static inline uint64_t rng_u64(rng_t* r, uint64_t idx) {
    uint64_t blk = idx >> 3;
    if (!r->valid || r->blk != blk) { chacha20_block(r->seed, r->stream, blk, r->w); r->blk = blk; r->valid = 1; }
    int o = (int)(idx & 7) * 2;
    return (uint64_t)r->w[o] | ((uint64_t)r->w[o + 1] << 32);
}
static inline rng_t rng_make(uint64_t seed, uint64_t stream) { rng_t r; r.seed = seed; r.stream = stream; r.blk = 0; r.valid = 0; return r; }

enum { STREAM_KSK_MASK = 1, STREAM_KSK_NOISE = 2, STREAM_BSK_MASK = 3, STREAM_BSK_NOISE = 4,
       STREAM_ENC_MASK = 5, STREAM_ENC_NOISE = 6 };

/* Box-Muller on two stream words; rounded to an integer number of 2^-64 torus units */
static int64_t gaussian(rng_t* r, uint64_t idx, double sigma) {
    uint64_t x1 = rng_u64(r, 2 * idx), x2 = rng_u64(r, 2 * idx + 1);
    double u1 = (double)((x1 >> 11) + 1) * 0x1.0p-53;
    double u2 = (double)(x2 >> 11) * 0x1.0p-53;
    double rad = sqrt(-2.0 * log(u1));
    double z = rad * cos(6.283185307179586 * u2);
    double scaled = z * (sigma * 18446744073709551616.0);
    return (int64_t)llround(scaled);
}

uint64_t or_rng_u64(uint64_t seed, uint64_t stream, uint64_t idx) { rng_t r = rng_make(seed, stream); return rng_u64(&r, idx); }
int64_t or_gaussian(uint64_t seed, uint64_t stream, uint64_t idx, double sigma) { rng_t r = rng_make(seed, stream); return gaussian(&r, idx, sigma); }

/* ------------------------------------------------- textbook negacyclic NTT */
typedef struct {
    int N, logN;
    uint64_t *psi, *psi_inv;  /* psi^i, psi^-i (i < N) */
    uint64_t *w, *w_inv;      /* omega^i (i < N/2), omega = psi^2 */
    uint64_t n_inv;
} ntt_plan;

static int ilog2(int x) { int l = 0; while ((1 << l) < x) l++; return l; }

static ntt_plan* ntt_plan_make(int N) {
    ntt_plan* P = (ntt_plan*)calloc(1, sizeof(ntt_plan));
    P->N = N; P->logN = ilog2(N);
    uint64_t psi = gl_pow(7, (GL_P - 1) / (2 * (uint64_t)N));
    uint64_t psi_inv = gl_pow(psi, 2 * (uint64_t)N - 1);
    P->psi = malloc(8 * N); P->psi_inv = malloc(8 * N); P->w = malloc(8 * N); P->w_inv = malloc(8 * N);
    uint64_t a = 1, b = 1;
    for (int i = 0; i < N; i++) { P->psi[i] = a; P->psi_inv[i] = b; a = gl_mul(a, psi); b = gl_mul(b, psi_inv); }
    uint64_t om = gl_mul(psi, psi), omi = gl_mul(psi_inv, psi_inv);
    a = 1; b = 1;
    for (int i = 0; i < N; i++) { P->w[i] = a; P->w_inv[i] = b; a = gl_mul(a, om); b = gl_mul(b, omi); }
    P->n_inv = gl_pow((uint64_t)N, GL_P - 2);
    return P;
}
static void ntt_plan_free(ntt_plan* P) { free(P->psi); free(P->psi_inv); free(P->w); free(P->w_inv); free(P); }

/* cyclic DIT NTT (bit-reverse, then butterflies) over w[] (forward) or w_inv[] */
static void cyclic_ntt(const ntt_plan* P, uint64_t* a, const uint64_t* w) {
    int N = P->N, L = P->logN;
    for (int i = 0; i < N; i++) {
        int r = 0;
        for (int b = 0; b < L; b++) if (i >> b & 1) r |= 1 << (L - 1 - b);
        if (i < r) { uint64_t t = a[i]; a[i] = a[r]; a[r] = t; }
    }
    for (int len = 2; len <= N; len <<= 1) {
        int step = N / len;
        for (int s = 0; s < N; s += len)
            for (int j = 0; j < len / 2; j++) {
                uint64_t u = a[s + j], v = gl_mul(a[s + j + len / 2], w[j * step]);
                a[s + j] = gl_add(u, v);
                a[s + j + len / 2] = gl_sub(u, v);
            }
    }
}
/* forward negacyclic transform: twist by psi^i then cyclic NTT */
static void nega_forward(const ntt_plan* P, uint64_t* a) {
    for (int i = 0; i < P->N; i++) a[i] = gl_mul(a[i], P->psi[i]);
    cyclic_ntt(P, a, P->w);
}
static void nega_inverse(const ntt_plan* P, uint64_t* a) {
    cyclic_ntt(P, a, P->w_inv);
    for (int i = 0; i < P->N; i++) a[i] = gl_mul(gl_mul(a[i], P->n_inv), P->psi_inv[i]);
}

void or_ring_mul(int N, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    ntt_plan* P = ntt_plan_make(N);
    uint64_t* x = malloc(8 * N); uint64_t* y = malloc(8 * N);
    memcpy(x, a, 8 * N); memcpy(y, b, 8 * N);
    nega_forward(P, x); nega_forward(P, y);
    for (int i = 0; i < N; i++) x[i] = gl_mul(x[i], y[i]);
    nega_inverse(P, x);
    memcpy(out, x, 8 * N);
    free(x); free(y); ntt_plan_free(P);
}
void or_ring_mul_schoolbook(int N, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    for (int i = 0; i < N; i++) out[i] = 0;
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) {
            uint64_t m = gl_mul(a[i], b[j]);
            int d = i + j;
            if (d < N) out[d] = gl_add(out[d], m);
            else out[d - N] = gl_sub(out[d - N], m);
        }
}

/* ------------------------------------------------ decompositions & maps */
/* PBS gadget (base 2^23, 1 level) in Z_p: g = floor(p / 2^23) = 2^41 - 2^9,
 * 2^23 * g = p - 1 = -1.  digit = round(x / g) in [0, 2^23], recentred to
 * [-2^22, 2^22); the wrap costs an error of exactly 1.  Returned in Z_p. */
uint64_t or_decompose_pbs(uint64_t x) {
    const uint64_t g = (1ULL << 41) - (1ULL << 9);
    uint64_t d = (uint64_t)(((u128)x + g / 2) / g);
    if (d >= (1ULL << 22)) return GL_P - ((1ULL << 23) - d); /* d - 2^23 < 0 */
    return d;
}

/* Z_p -> torus 2^64: round(x * 2^64 / p) */
uint64_t or_conv(uint64_t x) {
    u128 num = ((u128)x << 64) + (GL_P - 1) / 2;
    return (uint64_t)(num / GL_P);
}

/* signed base-2^B, L-level decomposition of the top B*L bits (rounded) */
static void ks_decompose(uint64_t a, int B, int L, int32_t* dig) {
    int bits = B * L;
    uint64_t c = (a >> (64 - bits)) + ((a >> (64 - bits - 1)) & 1);
    c &= (bits >= 64) ? ~0ULL : ((1ULL << bits) - 1);
    uint64_t mask = (1ULL << B) - 1, half = 1ULL << (B - 1);
    for (int j = L - 1; j >= 0; j--) {
        uint64_t d = c & mask;
        c >>= B;
        if (d >= half) { dig[j] = (int32_t)d - (int32_t)(1 << B); c += 1; }
        else dig[j] = (int32_t)d;
    }
}
void or_ks_decompose(uint64_t a, int B, int L, int32_t* dig) { ks_decompose(a, B, L, dig); }

static inline uint32_t mod_switch(uint64_t a, int log2N2) {
    return (uint32_t)((((a >> (64 - log2N2 - 1)) + 1) >> 1) & ((1ULL << log2N2) - 1));
}
uint32_t or_mod_switch(uint64_t a, int log2N2) { return mod_switch(a, log2N2); }

/* ------------------------------------------------------------- keygen */
void or_keygen_ksk(const or_params* P, const uint64_t* s_big, const uint64_t* s_small, uint64_t seed, uint64_t* ksk) {
    int big = P->k * P->N, n = P->n, L = P->ks_level, B = P->ks_base_log;
    rng_t rm = rng_make(seed, STREAM_KSK_MASK), rn = rng_make(seed, STREAM_KSK_NOISE);
    for (int i = 0; i < big; i++)
        for (int j = 0; j < L; j++) {
            uint64_t row = (uint64_t)i * L + j;
            uint64_t* o = ksk + row * (n + 1);
            uint64_t body = 0;
            for (int t = 0; t < n; t++) { o[t] = rng_u64(&rm, row * n + t); body += o[t] * s_small[t]; }
            int shift = 64 - B * (j + 1);
            body += s_big[i] << shift;
            body += (uint64_t)gaussian(&rn, row, P->lwe_sigma);
            o[n] = body;
        }
}

/* BSK in the coefficient domain mod p; layout [i][r][c][t], r,c in [0,k] */
void or_keygen_bsk(const or_params* P, const uint64_t* s_big, const uint64_t* s_small, uint64_t seed, uint64_t* bsk) {
    int k = P->k, N = P->N, n = P->n;
    const uint64_t g = (1ULL << 41) - (1ULL << 9);
    ntt_plan* NP = ntt_plan_make(N);
    /* NTT of the key polynomials S_j (coefficients of the flattened big key) */
    uint64_t* S = malloc(8 * (size_t)k * N);
    for (int j = 0; j < k; j++) {
        for (int t = 0; t < N; t++) S[(size_t)j * N + t] = s_big[(size_t)j * N + t];
        nega_forward(NP, S + (size_t)j * N);
    }
    rng_t rm = rng_make(seed, STREAM_BSK_MASK), rn = rng_make(seed, STREAM_BSK_NOISE);
    uint64_t* tmp = malloc(8 * (size_t)N);
    uint64_t* acc = malloc(8 * (size_t)N);
    for (int i = 0; i < n; i++)
        for (int r = 0; r <= k; r++) {
            uint64_t* row = bsk + ((size_t)i * (k + 1) + r) * (k + 1) * N;
            for (int t = 0; t < N; t++) acc[t] = 0;
            for (int j = 0; j < k; j++) {
                uint64_t* A = row + (size_t)j * N;
                uint64_t base = (((uint64_t)i * (k + 1) + r) * k + j) * N;
                for (int t = 0; t < N; t++) { uint64_t x = rng_u64(&rm, base + t); A[t] = x >= GL_P ? x - GL_P : x; }
                memcpy(tmp, A, 8 * (size_t)N);
                nega_forward(NP, tmp);
                for (int t = 0; t < N; t++) acc[t] = gl_add(acc[t], gl_mul(tmp[t], S[(size_t)j * N + t]));
            }
            nega_inverse(NP, acc);
            uint64_t* Bp = row + (size_t)k * N;
            uint64_t nb = ((uint64_t)i * (k + 1) + r) * N;
            for (int t = 0; t < N; t++) Bp[t] = gl_add(acc[t], gl_from_i64(gaussian(&rn, nb + t, P->glwe_sigma)));
            uint64_t mg = s_small[i] ? g : 0;
            row[(size_t)r * N] = gl_add(row[(size_t)r * N], mg);
        }
    free(tmp); free(acc); free(S); ntt_plan_free(NP);
}

/* ---------------------------------------------------- client encrypt/decrypt */
/* Encrypt block messages m in [0,16) (Delta = 2^59) under the big key, torus
 * 2^64.  Block q uses mask words q*kN.. and noise sample q of the seed's streams. */
void or_encrypt(const or_params* P, const uint64_t* s_big, const uint8_t* msgs, size_t count, uint64_t seed,
                uint64_t first_block, uint64_t* out) {
    int big = P->k * P->N;
    rng_t rm = rng_make(seed, STREAM_ENC_MASK), rn = rng_make(seed, STREAM_ENC_NOISE);
    for (size_t q = 0; q < count; q++) {
        uint64_t* o = out + q * (big + 1);
        uint64_t qb = first_block + q, body = 0;
        for (int t = 0; t < big; t++) { o[t] = rng_u64(&rm, qb * big + t); body += o[t] * s_big[t]; }
        body += (uint64_t)msgs[q] << 59;
        body += (uint64_t)gaussian(&rn, qb, P->glwe_sigma);
        o[big] = body;
    }
}
void or_phase(int dim, const uint64_t* s, const uint64_t* lwe, size_t count, uint64_t* phase) {
    for (size_t q = 0; q < count; q++) {
        const uint64_t* c = lwe + q * (dim + 1);
        uint64_t acc = c[dim];
        for (int t = 0; t < dim; t++) acc -= c[t] * s[t];
        phase[q] = acc;
    }
}
/* tfhe-rs shortint decrypt_message_and_carry: round(phase / Delta) mod 16 */
uint32_t or_decode16(uint64_t phase) {
    const uint64_t delta = 1ULL << 59;
    uint64_t rounding = (phase & (delta >> 1)) << 1;
    return (uint32_t)(((phase + rounding) / delta) % 16);
}

/* ------------------------------------------------------------ keyswitch */
void or_keyswitch(const or_params* P, const uint64_t* ksk, const uint64_t* in, size_t count, uint64_t* out) {
    int big = P->k * P->N, n = P->n, L = P->ks_level, B = P->ks_base_log;
    int32_t dig[64];
    for (size_t q = 0; q < count; q++) {
        const uint64_t* c = in + q * (big + 1);
        uint64_t* o = out + q * (n + 1);
        for (int t = 0; t < n; t++) o[t] = 0;
        o[n] = c[big];
        for (int i = 0; i < big; i++) {
            ks_decompose(c[i], B, L, dig);
            for (int j = 0; j < L; j++) {
                if (!dig[j]) continue;
                uint64_t d = (uint64_t)(int64_t)dig[j];
                const uint64_t* row = ksk + ((size_t)i * L + j) * (n + 1);
                for (int t = 0; t <= n; t++) o[t] -= d * row[t];
            }
        }
    }
}

/* --------------------------------------------------------- bootstrapping */
typedef struct {
    or_params P;
    ntt_plan* NP;
    uint64_t* bsk_ntt; /* [i][r][c][N] in the oracle's own NTT domain */
} or_bsk;

void* or_bsk_prepare(const or_params* P, const uint64_t* bsk) {
    or_bsk* K = (or_bsk*)calloc(1, sizeof(or_bsk));
    K->P = *P;
    K->NP = ntt_plan_make(P->N);
    size_t polys = (size_t)P->n * (P->k + 1) * (P->k + 1);
    K->bsk_ntt = malloc(8 * polys * P->N);
    memcpy(K->bsk_ntt, bsk, 8 * polys * P->N);
    #pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)polys; i++) nega_forward(K->NP, K->bsk_ntt + (size_t)i * P->N);
    return K;
}
void or_bsk_free(void* p) { or_bsk* K = (or_bsk*)p; ntt_plan_free(K->NP); free(K->bsk_ntt); free(K); }

/* LUT polynomial V (mod p): box = N/16 positions per message, recentred by half
 * a box; the last half box holds -f(0) (negacyclic wrap of message 16). */
static const uint64_t DELTA_P = (1ULL << 59) - (1ULL << 27); /* round(2^59 * p / 2^64) */
static void make_lut_poly(int N, const uint8_t lut[16], uint64_t* V) {
    int box = N / 16, half = box / 2;
    for (int j = 0; j < N; j++) {
        int m = (j + half) / box;
        if (m < 16) V[j] = (uint64_t)lut[m] * DELTA_P;
        else V[j] = lut[0] ? GL_P - (uint64_t)lut[0] * DELTA_P : 0;
    }
}
/* (X^a * poly)[j] for a in [0,2N), negacyclic */
static inline uint64_t rot_coef(const uint64_t* poly, int N, int j, int a) {
    int s = j - a;
    s %= 2 * N; if (s < 0) s += 2 * N;
    return s < N ? poly[s] : (poly[s - N] ? GL_P - poly[s - N] : 0);
}

/* Multi-value bootstrapping (Carpov, Izabachene, Mollimard, CT-RSA 2019):
 * with u(X) = sum_j X^j, u*(1-X) = 2 in Z[X]/(X^N+1), so every LUT polynomial
 * factors as V_f = (Delta/2) u * w_f where w_f is sparse with small integer
 * coefficients: f(m)-f(m-1) at m*box - box/2 (m = 1..15) and -(f(0)+f(15)) at
 * N - box/2.  One blind rotation of TV = (Delta_p/2) u then yields every LUT
 * on the same input: acc_f = w_f * acc (noise grows by ||w_f||_2).
 * "direct" jobs rotate V_f itself (one output, no w-step). */
int or_lut_terms(int N, const uint8_t lut[16], int32_t* pos, int32_t* d) {
    int box = N / 16, half = box / 2, n = 0;
    for (int m = 1; m < 16; m++) {
        int dd = (int)lut[m] - (int)lut[m - 1];
        if (dd) { pos[n] = m * box - half; d[n] = dd; n++; }
    }
    int dd = -((int)lut[0] + (int)lut[15]);
    if (dd) { pos[n] = N - half; d[n] = dd; n++; }
    return n;
}
/* sum_t d_t * (X^pos_t * poly)[j]  mod p */
static uint64_t apply_w(const uint64_t* poly, int N, int j, int nt, const int32_t* pos, const int32_t* d) {
    __int128 s = 0;
    for (int t = 0; t < nt; t++) {
        int src = j - pos[t];
        __int128 v;
        if (src >= 0) v = (__int128)poly[src];
        else v = -(__int128)poly[src + N];
        s += v * d[t];
    }
    s %= (__int128)GL_P;
    if (s < 0) s += GL_P;
    return (uint64_t)s;
}

/* Blind rotation of one keyswitched LWE, then for each of n_out LUTs the
 * w-step (unless direct), sample extract and Z_p -> 2^64 conversion. */
void or_blind_rotate_multi(void* pk, const uint64_t* ks_lwe, const uint8_t* luts, int n_out, int direct, uint64_t* outs) {
    or_bsk* K = (or_bsk*)pk;
    const or_params* P = &K->P;
    int k = P->k, N = P->N, n = P->n, log2N2 = ilog2(2 * N);
    size_t kp1 = (size_t)k + 1, big = (size_t)k * N;
    uint64_t* acc = calloc(kp1 * N, 8);
    uint64_t* D = malloc(8 * kp1 * N);
    uint64_t* res = malloc(8 * N);
    uint64_t* V = malloc(8 * N);
    /* direct == 1: the LUT polynomial itself; 0 (multi-value) and 2 (sign gate):
     * the constant test polynomial (Delta_p/2) * sum_j X^j */
    if (direct == 1) make_lut_poly(N, luts, V);
    else for (int j = 0; j < N; j++) V[j] = DELTA_P / 2;
    uint32_t b = mod_switch(ks_lwe[n], log2N2);
    /* acc = (0, X^{-b} V) */
    for (int j = 0; j < N; j++) acc[(size_t)k * N + j] = rot_coef(V, N, j, (2 * N - (int)b) % (2 * N));
    for (int i = 0; i < n; i++) {
        uint32_t a = mod_switch(ks_lwe[i], log2N2);
        if (a == 0) continue; /* X^0 acc - acc = 0: exactly a no-op */
        for (size_t c = 0; c < kp1; c++) {
            const uint64_t* A = acc + c * N;
            uint64_t* Dc = D + c * N;
            for (int j = 0; j < N; j++) Dc[j] = or_decompose_pbs(gl_sub(rot_coef(A, N, j, (int)a), A[j]));
            nega_forward(K->NP, Dc);
        }
        const uint64_t* G = K->bsk_ntt + (size_t)i * kp1 * kp1 * N;
        for (size_t c = 0; c < kp1; c++) {
            for (int t = 0; t < N; t++) {
                uint64_t s = 0;
                for (size_t r = 0; r < kp1; r++) s = gl_add(s, gl_mul(D[r * N + t], G[(r * kp1 + c) * N + t]));
                res[t] = s;
            }
            nega_inverse(K->NP, res);
            for (int t = 0; t < N; t++) acc[c * N + t] = gl_add(acc[c * N + t], res[t]);
        }
    }
    int32_t pos[17], d[17];
    for (int f = 0; f < (direct ? 1 : n_out); f++) {
        uint64_t* out = outs + (size_t)f * (big + 1);
        int nt = direct ? 0 : or_lut_terms(N, luts + 16 * f, pos, d);
        /* sample extract (coefficient 0) under the flattened key, then to 2^64 */
        for (int j = 0; j < k; j++) {
            const uint64_t* A = acc + (size_t)j * N;
            for (int t = 0; t < N; t++) {
                int src = t == 0 ? 0 : N - t;
                uint64_t a = direct ? A[src] : apply_w(A, N, src, nt, pos, d);
                uint64_t v = t == 0 ? a : (a ? GL_P - a : 0);
                out[(size_t)j * N + t] = or_conv(v);
            }
        }
        const uint64_t* B = acc + (size_t)k * N;
        out[big] = or_conv(direct ? B[0] : apply_w(B, N, 0, nt, pos, d));
        if (direct == 2) out[big] += 1ULL << 58; /* sign gate: +-Delta/2 + Delta/2 -> {0, Delta} */
    }
    free(acc); free(D); free(res); free(V);
}

/* single LUT, rotating the LUT polynomial itself */
void or_blind_rotate(void* pk, const uint64_t* ks_lwe, const uint8_t lut[16], uint64_t* out) {
    or_blind_rotate_multi(pk, ks_lwe, lut, 1, 1, out);
}

/* ------------------------------------------------------------------ gates */
/* A rotation job: c = offset*2^58 + sum_i w_i * in_i (mod 2^64), then one
 * blind rotation and n_out LUT outputs (direct: 0 multi-value, 1 the LUT
 * polynomial itself, 2 sign gate [c > 0]). */
typedef struct {
    int32_t n_in;
    int32_t offset;
    int32_t in_idx[16];
    int32_t in_w[16];
    int32_t n_out;
    int32_t direct;
    uint8_t lut[8][16];
} or_gate;

void or_lincomb(int big, const or_gate* g, const uint64_t* slots, uint64_t* out) {
    for (int t = 0; t <= big; t++) out[t] = 0;
    out[big] = (uint64_t)(int64_t)g->offset << 58;
    for (int q = 0; q < g->n_in; q++) {
        const uint64_t* x = slots + (size_t)g->in_idx[q] * (big + 1);
        uint64_t w = (uint64_t)(int64_t)g->in_w[q];
        for (int t = 0; t <= big; t++) out[t] += w * x[t];
    }
}

/* Evaluate `count` independent jobs over `slots` (LWE big, torus 2^64), OpenMP.
 * Outputs of job q start at out + out_first[q] * (kN+1). */
void or_gates(void* pk, const uint64_t* ksk, const or_gate* gates, size_t count, const uint64_t* slots,
              const int32_t* out_first, uint64_t* out) {
    or_bsk* K = (or_bsk*)pk;
    int big = K->P.k * K->P.N, n = K->P.n;
    #pragma omp parallel
    {
        uint64_t* lc = malloc(8 * (size_t)(big + 1));
        uint64_t* ks = malloc(8 * (size_t)(n + 1));
        #pragma omp for schedule(dynamic, 1)
        for (long q = 0; q < (long)count; q++) {
            or_lincomb(big, &gates[q], slots, lc);
            or_keyswitch(&K->P, ksk, lc, 1, ks);
            or_blind_rotate_multi(pk, ks, &gates[q].lut[0][0], gates[q].n_out, gates[q].direct,
                                  out + (size_t)out_first[q] * (big + 1));
        }
        free(lc); free(ks);
    }
}

int or_num_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}
void or_set_threads(int t) {
#ifdef _OPENMP
    extern void omp_set_num_threads(int);
    omp_set_num_threads(t);
#else
    (void)t;
#endif
}
