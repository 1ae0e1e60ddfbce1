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
 * n=742, k=1, N=2048, PBS 2^23 x 1, KS 2^3 x 5, Delta = 2^59).  Two GLWE/GGSW
 * rings, as in the product (fheregex.h FR_RING_*):
 *  - the torus ring (default): the 2^64 torus with an f64 negacyclic FFT,
 *    tfhe-rs's own arithmetic class (concrete-fft 0.1.0, reference
 *    Cargo.lock:110-114), restated from the operation sequence specified in
 *    the product's csrc/fft.h (floating point is not associative: bit-identity
 *    needs the same sequence); and, independently of that sequence, the same
 *    unrolled ladder in exact u64 arithmetic (blind_rotate_exact: schoolbook
 *    negacyclic products mod 2^64), the yardstick the f64 ladder is held to
 *    (tests/test_exact_br.py);
 *  - the RNS ring: Z_Q[X]/(X^N+1) with Q = 998244353 * 1004535809 (~2^59.8,
 *    exact integer NTTs per prime + CRT); sample-extracted LWEs are mapped back
 *    to the 2^64 torus by x -> sum_i round(2^64 * u_i / p_i) (u_i = x * (Q/p_i)^-1
 *    mod p_i, which is round(x * 2^64 / Q) up to one unit).
 * Every ciphertext that crosses the boundary decrypts with the reference's
 * client key and the tfhe-rs decoding rule (shortint decrypt_message_and_carry).
 *
 * Call sites in the reference this path replaces: src/regex/execution.rs:76,
 * 93,110,143,173,190 (smart_eq/gt/le/bitand/bitor/bitxor), trivial constants
 * src/regex/ciphertext.rs:8-30, keygen src/regex/ciphertext.rs:42-45 and
 * engine.rs:252 (ServerKey::new).
 *
 * Parity pins: the fixture client key (decoding verified in tests), the 25
 * decrypted-result cases of src/regex/engine.rs:256-280, and bit-identity with
 * the GPU path (same keys, same inputs).  The ring product here is a textbook
 * twisted cyclic NTT per prime with 64-bit '%' arithmetic and a 128-bit CRT,
 * written independently of the GPU's lazy Montgomery merged-psi NTT; both are
 * exact in Z_Q so the products agree bit for bit.  Likewise the boundary maps
 * (gadget digit, Z_Q -> torus) use plain 128-bit division here and
 * reciprocal/Montgomery forms on the GPU.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* RNS ring: Q = p0 * p1 */
static const uint64_t PR[2] = {998244353ULL, 1004535809ULL};
#define Q_MOD (998244353ULL * 1004535809ULL)

/* ---------------------------------------------------------------- params */
typedef struct {
    int32_t k;            /* GLWE dimension */
    int32_t N;            /* polynomial size */
    int32_t n;            /* small LWE dimension */
    int32_t ks_base_log;  /* 3 */
    int32_t ks_level;     /* 5 */
    int32_t pbs_base_log; /* 23 */
    int32_t pbs_level;    /* 1 */
    int32_t ring;         /* 0: Z_Q RNS NTT ring, 1: torus 2^64 + f64 FFT */
    double lwe_sigma;     /* KSK noise (std dev as a fraction of the torus) */
    double glwe_sigma;    /* BSK / fresh-encryption noise */
} or_params;

/* ------------------------------------------------------------ Z_Q, Z_p */
static inline uint64_t q_add(uint64_t a, uint64_t b) { uint64_t s = a + b; return s >= Q_MOD ? s - Q_MOD : s; }
static inline uint64_t q_sub(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (Q_MOD - b); }
static inline uint64_t q_neg(uint64_t a) { return a ? Q_MOD - a : 0; }
static inline uint64_t q_mul(uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) % Q_MOD); }
static inline uint64_t q_from_i64(int64_t v) { return v >= 0 ? (uint64_t)v % Q_MOD : q_neg((uint64_t)(-v) % Q_MOD); }
static uint64_t pm_pow(uint64_t b, uint64_t e, uint64_t p) {
    uint64_t r = 1;
    b %= p;
    while (e) { if (e & 1) r = r * b % p; b = b * b % p; e >>= 1; }
    return r;
}
/* CRT of residues r0 mod p0, r1 mod p1 -> [0, Q) */
static inline uint64_t crt2(uint64_t r0, uint64_t r1) {
    static uint64_t inv = 0;
    if (!inv) inv = pm_pow(PR[0], PR[1] - 2, PR[1]);
    uint64_t k = (r1 + PR[1] - r0 % PR[1]) % PR[1] * inv % PR[1];
    return r0 + PR[0] * k;
}

uint64_t or_q_mul(uint64_t a, uint64_t b) { return q_mul(a, b); }
uint64_t or_q_modulus(void) { return Q_MOD; }

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

/* Box-Muller on two stream words; z * sigma * scale rounded to an integer
 * (scale 2^64: torus units; scale Q: units of Z_Q) */
#define TORUS_SCALE 18446744073709551616.0
static int64_t gaussian_s(rng_t* r, uint64_t idx, double sigma, double scale) {
    uint64_t x1 = rng_u64(r, 2 * idx), x2 = rng_u64(r, 2 * idx + 1);
    double u1 = (double)((x1 >> 11) + 1) * 0x1.0p-53;
    double u2 = (double)(x2 >> 11) * 0x1.0p-53;
    double rad = sqrt(-2.0 * log(u1));
    double z = rad * cos(6.283185307179586 * u2);
    double scaled = z * (sigma * scale);
    return (int64_t)llround(scaled);
}
static int64_t gaussian(rng_t* r, uint64_t idx, double sigma) { return gaussian_s(r, idx, sigma, TORUS_SCALE); }

uint64_t or_rng_u64(uint64_t seed, uint64_t stream, uint64_t idx) { rng_t r = rng_make(seed, stream); return rng_u64(&r, idx); }
int64_t or_gaussian(uint64_t seed, uint64_t stream, uint64_t idx, double sigma) { rng_t r = rng_make(seed, stream); return gaussian(&r, idx, sigma); }

/* ------------------------------------------- textbook negacyclic NTT mod p */
typedef struct {
    int N, logN;
    uint64_t *psi[2], *psi_inv[2];  /* psi^i, psi^-i (i < N) per prime */
    uint64_t *w[2], *w_inv[2];      /* omega^i, omega = psi^2 */
    uint64_t n_inv[2];
} ntt_plan;

static int ilog2(int x) { int l = 0; while ((1 << l) < x) l++; return l; }

static ntt_plan* ntt_plan_make(int N) {
    ntt_plan* P = (ntt_plan*)calloc(1, sizeof(ntt_plan));
    P->N = N; P->logN = ilog2(N);
    for (int q = 0; q < 2; q++) {
        uint64_t p = PR[q];
        uint64_t psi = pm_pow(3, (p - 1) / (2 * (uint64_t)N), p); /* 3 generates Z_p^* */
        uint64_t psi_inv = pm_pow(psi, p - 2, p);
        P->psi[q] = malloc(8 * N); P->psi_inv[q] = malloc(8 * N); P->w[q] = malloc(8 * N); P->w_inv[q] = malloc(8 * N);
        uint64_t a = 1, b = 1;
        for (int i = 0; i < N; i++) { P->psi[q][i] = a; P->psi_inv[q][i] = b; a = a * psi % p; b = b * psi_inv % p; }
        uint64_t om = psi * psi % p, omi = psi_inv * psi_inv % p;
        a = 1; b = 1;
        for (int i = 0; i < N; i++) { P->w[q][i] = a; P->w_inv[q][i] = b; a = a * om % p; b = b * omi % p; }
        P->n_inv[q] = pm_pow((uint64_t)N, p - 2, p);
    }
    return P;
}
static void ntt_plan_free(ntt_plan* P) {
    for (int q = 0; q < 2; q++) { free(P->psi[q]); free(P->psi_inv[q]); free(P->w[q]); free(P->w_inv[q]); }
    free(P);
}

/* cyclic DIT NTT mod p (bit-reverse, then butterflies) over w[] or w_inv[] */
static void cyclic_ntt(const ntt_plan* P, uint64_t p, uint64_t* a, const uint64_t* w) {
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
                uint64_t u = a[s + j], v = a[s + j + len / 2] * w[j * step] % p;
                a[s + j] = (u + v) % p;
                a[s + j + len / 2] = (u + p - v) % p;
            }
    }
}
/* forward negacyclic transform mod PR[q]: twist by psi^i then cyclic NTT */
static void nega_forward(const ntt_plan* P, int q, uint64_t* a) {
    uint64_t p = PR[q];
    for (int i = 0; i < P->N; i++) a[i] = a[i] % p * P->psi[q][i] % p;
    cyclic_ntt(P, p, a, P->w[q]);
}
static void nega_inverse(const ntt_plan* P, int q, uint64_t* a) {
    uint64_t p = PR[q];
    cyclic_ntt(P, p, a, P->w_inv[q]);
    for (int i = 0; i < P->N; i++) a[i] = a[i] * P->n_inv[q] % p * P->psi_inv[q][i] % p;
}

/* negacyclic product mod Q of a, b in [0, Q) */
static void ring_mul_q(const ntt_plan* P, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    int N = P->N;
    uint64_t* x[2]; uint64_t* y = malloc(8 * N);
    for (int q = 0; q < 2; q++) {
        x[q] = malloc(8 * N);
        for (int i = 0; i < N; i++) { x[q][i] = a[i] % PR[q]; y[i] = b[i] % PR[q]; }
        nega_forward(P, q, x[q]); nega_forward(P, q, y);
        for (int i = 0; i < N; i++) x[q][i] = x[q][i] * y[i] % PR[q];
        nega_inverse(P, q, x[q]);
    }
    for (int i = 0; i < N; i++) out[i] = crt2(x[0][i], x[1][i]);
    free(x[0]); free(x[1]); free(y);
}
void or_ring_mul(int N, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    ntt_plan* P = ntt_plan_make(N);
    ring_mul_q(P, a, b, out);
    ntt_plan_free(P);
}
void or_ring_mul_schoolbook(int N, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    for (int i = 0; i < N; i++) out[i] = 0;
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) {
            uint64_t m = q_mul(a[i], b[j]);
            int d = i + j;
            if (d < N) out[d] = q_add(out[d], m);
            else out[d - N] = q_sub(out[d - N], m);
        }
}

/* ------------------------------------------- f64 negacyclic FFT (torus ring)
 * Restatement of the product's FR_RING_FFT transform (fhe-regex_amd/csrc/fft.h,
 * which documents the derivation): tfhe-rs 0.2 multiplies GGSW x GLWE through
 * an f64 FFT of the folded polynomial (concrete-fft 0.1.0, reference
 * Cargo.lock:110-114).  A real polynomial a of degree < N folds into M = N/2
 * complex points z_k = a_k + i a_(k+M) (a mod x^M - i); the merged-twiddle
 * split of x^M - i evaluates it at psi^L(j) (psi = e^(i pi/N)).  Because the
 * result is floating point, parity with the GPU is bit-exact only if the same
 * IEEE-754 operation sequence is used: the butterflies, complex products and
 * the f64 -> torus map below are written to that specification (fma where the
 * specification fuses, -ffp-contract=off elsewhere).  Independent checks of
 * the transform itself (against exact integer products) live in tests/. */
typedef struct { double re, im; } cplx;
static inline void c_mul(double ar, double ai, double br, double bi, double* zr, double* zi) {
    double pr = -(ai * bi), pi = ai * br;
    *zr = fma(ar, br, pr);
    *zi = fma(ar, bi, pi);
}
static inline void c_mac(double ar, double ai, double br, double bi, double* zr, double* zi) {
    *zr = fma(-ai, bi, fma(ar, br, *zr));
    *zi = fma(ai, br, fma(ar, bi, *zi));
}
static inline void quarter_turns(double ar, double ai, uint32_t q, double* zr, double* zi) {
    if (q & 1) { double t = ar; ar = -ai; ai = t; }
    if (q & 2) { ar = -ar; ai = -ai; }
    *zr = ar; *zi = ai;
}
/* psi^x = i^q (cos(pi r/N), sin(pi r/N)), x = q N/2 + r (mod 2N) */
static cplx psi_pow(int N, long x) {
    long twoN = 2L * N, quarter = N / 2;
    x %= twoN; if (x < 0) x += twoN;
    uint32_t q = (uint32_t)(x / quarter);
    long r = x % quarter;
    double ang = (double)r * (3.14159265358979323846 / (double)N);
    cplx z;
    quarter_turns(cos(ang), sin(ang), q, &z.re, &z.im);
    return z;
}
typedef struct { int N, M, LOG; cplx* tw; cplx* qt; uint16_t* leaf; } fft_plan;
static fft_plan* fft_plan_make(int N) {
    fft_plan* F = (fft_plan*)calloc(1, sizeof(fft_plan));
    F->N = N; F->M = N / 2; F->LOG = ilog2(N / 2);
    F->tw = calloc(F->M, sizeof(cplx)); F->qt = malloc(sizeof(cplx) * (N / 2)); F->leaf = malloc(2 * F->M);
    for (int r = 0; r < N / 2; r++) F->qt[r] = psi_pow(N, r);
    /* split-tree exponents: E(0,0) = M; children E/2 and E/2 + N; twiddle psi^(E/2) */
    long* E = malloc(sizeof(long) * F->M);
    long* nx = malloc(sizeof(long) * F->M);
    E[0] = F->M;
    for (int s = 0; s < F->LOG; s++) {
        for (int b = 0; b < (1 << s); b++) {
            F->tw[(1 << s) + b] = psi_pow(N, E[b] / 2);
            nx[2 * b] = (E[b] / 2) % (2L * N);
            nx[2 * b + 1] = (E[b] / 2 + N) % (2L * N);
        }
        long* t = E; E = nx; nx = t;
    }
    for (int j = 0; j < F->M; j++) F->leaf[j] = (uint16_t)E[j];
    free(E); free(nx);
    return F;
}
static void fft_plan_free(fft_plan* F) { free(F->tw); free(F->qt); free(F->leaf); free(F); }
/* forward: (lo, hi) -> (lo + c hi, lo - c hi), natural order -> slot order;
 * lo + c hi as two nested fmas per component, lo - c hi as 2 lo - (lo + c hi) */
static void fft_forward(const fft_plan* F, cplx* z) {
    for (int s = 0; s < F->LOG; s++) {
        int h = F->M >> (s + 1);
        for (int b = 0; b < (1 << s); b++) {
            cplx c = F->tw[(1 << s) + b];
            for (int j = b * 2 * h; j < b * 2 * h + h; j++) {
                double xr = z[j].re, xi = z[j].im, yr = z[j + h].re, yi = z[j + h].im;
                double ur = fma(c.re, yr, fma(-c.im, yi, xr));
                double ui = fma(c.re, yi, fma(c.im, yr, xi));
                z[j + h].re = fma(2.0, xr, -ur); z[j + h].im = fma(2.0, xi, -ui);
                z[j].re = ur; z[j].im = ui;
            }
        }
    }
}
/* inverse radix-4 group (fft.h inv_r4): stages s1 = 2p + 1 then s0 = 2p on x0..x3
 * (x1 = x0's stage-s1 partner, x2 its stage-s0 partner); stage s1's twiddles are ca
 * and i ca (exactly: split-tree siblings), stage s0's c:
 *   a = x0 + x1, d1 = x0 - x1, b = x2 + x3, d2 = x2 - x3, t1 = d1 - i d2, t2 = d1 + i d2,
 *   x0 <- a + b, x1 <- conj(ca) t1, x2 <- conj(c) (a - b), x3 <- conj(c ca) t2 */
static inline void conj_mul(double wr, double wi, double dr, double di, double* zr, double* zi) {
    *zr = fma(wr, dr, wi * di);
    *zi = fma(wr, di, -(wi * dr));
}
static void inv_r4(cplx* x0, cplx* x1, cplx* x2, cplx* x3, cplx c, cplx ca, cplx cc) {
    double ar = x0->re + x1->re, ai = x0->im + x1->im, d1r = x0->re - x1->re, d1i = x0->im - x1->im;
    double br = x2->re + x3->re, bi = x2->im + x3->im, d2r = x2->re - x3->re, d2i = x2->im - x3->im;
    double t1r = d1r + d2i, t1i = d1i - d2r, t2r = d1r - d2i, t2i = d1i + d2r;
    double er = ar - br, ei = ai - bi;
    x0->re = ar + br; x0->im = ai + bi;
    conj_mul(ca.re, ca.im, t1r, t1i, &x1->re, &x1->im);
    conj_mul(c.re, c.im, er, ei, &x2->re, &x2->im);
    conj_mul(cc.re, cc.im, t2r, t2i, &x3->re, &x3->im);
}
/* inverse: (A, B) -> (A + B, conj(c) (A - B)), slot order -> natural, times M;
 * for even log2 M the stages go in radix-4 pairs (2p + 1, 2p) */
static void fft_inverse(const fft_plan* F, cplx* z) {
    if (F->LOG % 2 == 0) {
        for (int s0 = F->LOG - 2; s0 >= 0; s0 -= 2) {
            int s1 = s0 + 1, h1 = F->M >> (s1 + 1), h0 = 2 * h1;
            for (int b = 0; b < (1 << s0); b++) {
                cplx c = F->tw[(1 << s0) + b], ca = F->tw[(1 << s1) + 2 * b], cc;
                c_mul(c.re, c.im, ca.re, ca.im, &cc.re, &cc.im);
                for (int j = b * 2 * h0; j < b * 2 * h0 + h1; j++)
                    inv_r4(&z[j], &z[j + h1], &z[j + h0], &z[j + h0 + h1], c, ca, cc);
            }
        }
        return;
    }
    for (int s = F->LOG - 1; s >= 0; s--) {
        int h = F->M >> (s + 1);
        for (int b = 0; b < (1 << s); b++) {
            cplx c = F->tw[(1 << s) + b];
            for (int j = b * 2 * h; j < b * 2 * h + h; j++) {
                double ur = z[j].re, ui = z[j].im, vr = z[j + h].re, vi = z[j + h].im;
                double dr = ur - vr, di = ui - vi;
                z[j].re = ur + vr; z[j].im = ui + vi;
                double pr = c.im * di, pi = -(c.im * dr);
                z[j + h].re = fma(c.re, dr, pr);
                z[j + h].im = fma(c.re, di, pi);
            }
        }
    }
}
/* f64 (integer-valued, |v| < 2^100) -> v mod 2^64, exact */
static inline uint64_t torus_of(double v) {
    double k = nearbyint(v * 0x1p-64);
    double ri = nearbyint(fma(-k, 0x1p64, v));
    double hi = floor(ri * 0x1p-32);
    double lo = fma(-hi, 0x1p32, ri);
    double hu = hi < 0 ? hi + 0x1p32 : hi;
    return ((uint64_t)(uint32_t)hu << 32) + (uint64_t)(uint32_t)lo;
}
/* f64 blind-rotation accumulator (fft.h): a torus value held as a double in
 * [-2^63, 2^63]; digit rint(a 2^-(64-B)); update reduce(a + v) with
 * reduce(a) = fma(-rint(a 2^-64), 2^64, a) (exact) */
static inline double acc_digit(double a, int B) { return nearbyint(a * ldexp(1.0, B - 64)); }
static inline double acc_reduce(double a) { return fma(-nearbyint(a * 0x1p-64), 0x1p64, a); }
/* negacyclic product mod 2^64 through the FFT (test hook: b must be small,
 * |b| * |a| * N < 2^50, for an exact result) and exactly (schoolbook) */
void or_fft_ring_mul(int N, const int64_t* a, const int64_t* b, int64_t* out) {
    fft_plan* F = fft_plan_make(N);
    int M = N / 2;
    cplx* x = malloc(sizeof(cplx) * M); cplx* y = malloc(sizeof(cplx) * M);
    for (int k = 0; k < M; k++) { x[k].re = (double)a[k]; x[k].im = (double)a[k + M]; y[k].re = (double)b[k]; y[k].im = (double)b[k + M]; }
    fft_forward(F, x); fft_forward(F, y);
    for (int k = 0; k < M; k++) { double zr, zi; c_mul(x[k].re, x[k].im, y[k].re, y[k].im, &zr, &zi); x[k].re = zr * ldexp(1.0, -F->LOG); x[k].im = zi * ldexp(1.0, -F->LOG); }
    fft_inverse(F, x);
    for (int k = 0; k < M; k++) { out[k] = (int64_t)torus_of(x[k].re); out[k + M] = (int64_t)torus_of(x[k].im); }
    free(x); free(y); fft_plan_free(F);
}
void or_fft_tables(int N, double* tw, double* qt, uint16_t* leaf) {
    fft_plan* F = fft_plan_make(N);
    memcpy(tw, F->tw, sizeof(cplx) * F->M); memcpy(qt, F->qt, sizeof(cplx) * (N / 2)); memcpy(leaf, F->leaf, 2 * F->M);
    fft_plan_free(F);
}
uint64_t or_torus_of(double v) { return torus_of(v); }

/* ------------------------------------------------ decompositions & maps */
/* PBS gadget (base 2^23, 1 level) in Z_Q: g = round(Q / 2^23).  Digit of x:
 * write x = r0 + p0 * k (r0 = x mod p0, k = (x - r0) / p0 < p1), take
 * t = (k * M + 2^37) >> 38 with M = round(2^61 / p1) (t ~ x * 2^23 / Q in
 * [0, 2^23]) and recentre to [-2^22, 2^22).  Returned as int64. */
static uint64_t pbs_g(void) { return (Q_MOD + (1ULL << 22)) >> 23; }
static int64_t decompose_q(uint64_t x) {
    const uint64_t p1 = PR[1];
    const uint64_t M = ((1ULL << 61) + p1 / 2) / p1;
    const uint64_t k = (x - x % PR[0]) / PR[0];
    const uint64_t t = (uint64_t)(((u128)k * M + ((u128)1 << 37)) >> 38);
    return t >= (1ULL << 22) ? (int64_t)t - (1LL << 23) : (int64_t)t;
}
uint64_t or_decompose_pbs(uint64_t x) { return (uint64_t)decompose_q(x); }
uint64_t or_pbs_gadget(void) { return pbs_g(); }

/* Z_Q -> torus 2^64 from the residues: sum_i round(2^64 * u_i / p_i) mod 2^64,
 * u_i = x * (Q/p_i)^-1 mod p_i (CRT: sum_i u_i/p_i = x/Q mod 1). */
uint64_t or_conv(uint64_t x) {
    uint64_t y = 0;
    for (int q = 0; q < 2; q++) {
        uint64_t p = PR[q], other = PR[1 - q];
        uint64_t u = x % p * pm_pow(other, p - 2, p) % p;
        y += (uint64_t)((((u128)u << 64) + (p - 1) / 2) / p);
    }
    return y;
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

/* Bootstrapping-key unrolling (pairs of LWE coefficients per blind-rotation
 * step; k = 1 on both rings, every k on the torus ring -- the product's
 * Params::bsk_unroll): GGSW number w = 3t + g encrypts, for i = 2t, j = 2t+1,
 *   g = 0: s_i s_j,  g = 1: s_i (1 - s_j),  g = 2: (1 - s_i) s_j
 * (s_j = 0 past the end), so that X^(a_i s_i + a_j s_j) - 1 =
 * sum_g m_g (X^(e_g) - 1) with e = (a_i + a_j, a_i, a_j).  RNS ring, k > 1:
 * one GGSW of s_i per coefficient (no unrolling). */
static int bsk_unroll(const or_params* P) { return (P->k == 1 || P->ring == 1) ? 2 : 1; }
static size_t bsk_ggsw(const or_params* P) {
    return bsk_unroll(P) == 2 ? 3 * (size_t)((P->n + 1) / 2) : (size_t)P->n;
}
size_t or_bsk_len(const or_params* P) { return bsk_ggsw(P) * (size_t)(P->k + 1) * (P->k + 1) * P->N; }
int or_bsk_unroll(const or_params* P) { return bsk_unroll(P); }
static uint64_t ggsw_msg(const or_params* P, const uint64_t* s_small, size_t w) {
    if (bsk_unroll(P) == 1) return s_small[w];
    size_t t = w / 3, g = w % 3, i = 2 * t, j = 2 * t + 1;
    uint64_t si = s_small[i], sj = j < (size_t)P->n ? s_small[j] : 0;
    return g == 0 ? (si & sj) : g == 1 ? (si & (1 - sj)) : ((1 - si) & sj);
}

/* BSK in the coefficient domain mod Q; layout [w][r][c][t], r,c in [0,k].
 * GGSW row r of message m_w: a GLWE encryption of zero (mask uniform in Z_Q,
 * body = sum_j A_j S_j + e) plus g * m_w on component r. */
/* Torus ring: row r of GGSW w is a GLWE encryption of zero on the 2^64 torus
 * (mask uniform u64, body = sum_j A_j S_j + e) plus m_w 2^(64-B) on
 * coefficient 0 of component r (one-level gadget, B = pbs_base_log); the
 * negacyclic products with the binary key are summed exactly. */
static void keygen_bsk_torus(const or_params* P, const uint64_t* s_big, const uint64_t* s_small, uint64_t seed, uint64_t* bsk) {
    int k = P->k, N = P->N;
    const size_t nw = bsk_ggsw(P), kp1 = (size_t)k + 1;
    const uint64_t gadget = 1ULL << (64 - P->pbs_base_log);
    #pragma omp parallel for schedule(dynamic, 4)
    for (long i = 0; i < (long)nw; i++) {
        rng_t rm = rng_make(seed, STREAM_BSK_MASK), rn = rng_make(seed, STREAM_BSK_NOISE);
        for (size_t r = 0; r < kp1; r++) {
            uint64_t* row = bsk + ((size_t)i * kp1 + r) * kp1 * N;
            uint64_t* B = row + (size_t)k * N;
            for (int t = 0; t < N; t++) B[t] = 0;
            for (int j = 0; j < k; j++) {
                uint64_t* A = row + (size_t)j * N;
                uint64_t base = (((uint64_t)i * kp1 + r) * k + j) * N;
                for (int t = 0; t < N; t++) A[t] = rng_u64(&rm, base + t);
                const uint64_t* S = s_big + (size_t)j * N;
                for (int t = 0; t < N; t++) {
                    if (!A[t]) continue;
                    for (int u = 0; u < N; u++) {
                        if (!S[u]) continue;
                        if (t + u < N) B[t + u] += A[t]; else B[t + u - N] -= A[t];
                    }
                }
            }
            uint64_t nb = ((uint64_t)i * kp1 + r) * N;
            for (int t = 0; t < N; t++) B[t] += (uint64_t)gaussian(&rn, nb + t, P->glwe_sigma);
            if (ggsw_msg(P, s_small, i)) row[r * N] += gadget;
        }
    }
}

void or_keygen_bsk(const or_params* P, const uint64_t* s_big, const uint64_t* s_small, uint64_t seed, uint64_t* bsk) {
    if (P->ring == 1) { keygen_bsk_torus(P, s_big, s_small, seed, bsk); return; }
    int k = P->k, N = P->N;
    const uint64_t g = pbs_g();
    const size_t nw = bsk_ggsw(P);
    ntt_plan* NP = ntt_plan_make(N);
    rng_t rm = rng_make(seed, STREAM_BSK_MASK), rn = rng_make(seed, STREAM_BSK_NOISE);
    uint64_t* prod = malloc(8 * (size_t)N);
    uint64_t* acc = malloc(8 * (size_t)N);
    for (size_t i = 0; i < nw; i++)
        for (int r = 0; r <= k; r++) {
            uint64_t* row = bsk + ((size_t)i * (k + 1) + r) * (k + 1) * N;
            for (int t = 0; t < N; t++) acc[t] = 0;
            for (int j = 0; j < k; j++) {
                uint64_t* A = row + (size_t)j * N;
                uint64_t base = (((uint64_t)i * (k + 1) + r) * k + j) * N;
                for (int t = 0; t < N; t++) A[t] = (uint64_t)(((u128)rng_u64(&rm, base + t) * Q_MOD) >> 64);
                ring_mul_q(NP, A, s_big + (size_t)j * N, prod);
                for (int t = 0; t < N; t++) acc[t] = q_add(acc[t], prod[t]);
            }
            uint64_t* Bp = row + (size_t)k * N;
            uint64_t nb = ((uint64_t)i * (k + 1) + r) * N;
            for (int t = 0; t < N; t++)
                Bp[t] = q_add(acc[t], q_from_i64(gaussian_s(&rn, nb + t, P->glwe_sigma, (double)Q_MOD)));
            if (ggsw_msg(P, s_small, i)) row[(size_t)r * N] = q_add(row[(size_t)r * N], g);
        }
    free(prod); free(acc); ntt_plan_free(NP);
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
    uint64_t* bsk_ntt[2]; /* [i][r][c][N] residues mod p_q in the oracle's own NTT domain */
    fft_plan* FP;         /* torus ring */
    cplx* bsk_f;          /* [i][r][c][M] Fourier domain, scaled by 1/M */
} or_bsk;

void* or_bsk_prepare(const or_params* P, const uint64_t* bsk) {
    or_bsk* K = (or_bsk*)calloc(1, sizeof(or_bsk));
    K->P = *P;
    if (P->ring == 1) {
        if (P->k + 1 > 8) { free(K); return NULL; }
        K->FP = fft_plan_make(P->N);
        int M = P->N / 2;
        size_t polys = bsk_ggsw(P) * (P->k + 1) * (P->k + 1);
        K->bsk_f = malloc(sizeof(cplx) * polys * M);
        double sc = ldexp(1.0, -K->FP->LOG);
        #pragma omp parallel for schedule(static)
        for (long i = 0; i < (long)polys; i++) {
            const uint64_t* a = bsk + (size_t)i * P->N;
            cplx* z = K->bsk_f + (size_t)i * M;
            for (int t = 0; t < M; t++) { z[t].re = (double)(int64_t)a[t]; z[t].im = (double)(int64_t)a[t + M]; }
            fft_forward(K->FP, z);
            for (int t = 0; t < M; t++) { z[t].re *= sc; z[t].im *= sc; }
        }
        return K;
    }
    K->NP = ntt_plan_make(P->N);
    size_t polys = bsk_ggsw(P) * (P->k + 1) * (P->k + 1);
    for (int q = 0; q < 2; q++) {
        K->bsk_ntt[q] = malloc(8 * polys * P->N);
        memcpy(K->bsk_ntt[q], bsk, 8 * polys * P->N);
        #pragma omp parallel for schedule(static)
        for (long i = 0; i < (long)polys; i++) nega_forward(K->NP, q, K->bsk_ntt[q] + (size_t)i * P->N);
    }
    return K;
}
void or_bsk_free(void* p) {
    or_bsk* K = (or_bsk*)p;
    if (K->FP) { fft_plan_free(K->FP); free(K->bsk_f); free(K); return; }
    ntt_plan_free(K->NP); free(K->bsk_ntt[0]); free(K->bsk_ntt[1]); free(K);
}
/* Fourier-domain BSK (test hook: the product's host transform must agree bit for bit) */
void or_bsk_fourier(void* pk, double* out) {
    or_bsk* K = (or_bsk*)pk;
    size_t polys = bsk_ggsw(&K->P) * (K->P.k + 1) * (K->P.k + 1);
    memcpy(out, K->bsk_f, sizeof(cplx) * polys * (K->P.N / 2));
}

/* Delta = 2^59 on the torus is D_Q = 2 * round(Q / 64) in Z_Q */
static uint64_t half_delta_q(void) { return (Q_MOD + 32) / 64; }
/* LUT polynomial V (mod Q): box = N/16 positions per message, recentred by half
 * a box; the last half box holds -f(0) (negacyclic wrap of message 16). */
static void make_lut_poly(int N, const uint8_t lut[16], uint64_t* V) {
    const uint64_t dq = 2 * half_delta_q();
    int box = N / 16, half = box / 2;
    for (int j = 0; j < N; j++) {
        int m = (j + half) / box;
        if (m < 16) V[j] = (uint64_t)lut[m] * dq;
        else V[j] = q_neg((uint64_t)lut[0] * dq);
    }
}
/* (X^a * poly)[j] for a in [0,2N), negacyclic */
static inline uint64_t rot_coef(const uint64_t* poly, int N, int j, int a) {
    int s = j - a;
    s %= 2 * N; if (s < 0) s += 2 * N;
    return s < N ? poly[s] : q_neg(poly[s - N]);
}

/* Multi-value bootstrapping (Carpov, Izabachene, Mollimard, CT-RSA 2019):
 * with u(X) = sum_j X^j, u*(1-X) = 2 in Z[X]/(X^N+1), so every LUT polynomial
 * factors as V_f = (Delta/2) u * w_f where w_f is sparse with small integer
 * coefficients: f(m)-f(m-1) at m*box - box/2 (m = 1..15) and -(f(0)+f(15)) at
 * N - box/2.  One blind rotation of TV = (Delta/2) u then yields every LUT
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
/* sum_t d_t * (X^pos_t * poly)[j]  mod Q */
static uint64_t apply_w(const uint64_t* poly, int N, int j, int nt, const int32_t* pos, const int32_t* d) {
    __int128 s = 0;
    for (int t = 0; t < nt; t++) {
        int src = j - pos[t];
        __int128 v;
        if (src >= 0) v = (__int128)poly[src];
        else v = -(__int128)poly[src + N];
        s += v * d[t];
    }
    s %= (__int128)Q_MOD;
    if (s < 0) s += Q_MOD;
    return (uint64_t)s;
}

/* Blind rotation of one keyswitched LWE, then for each of n_out LUTs the
 * w-step (unless direct), sample extract and Z_Q -> 2^64 conversion. */
/* Torus ring: the unrolled blind rotation with the three Fourier GGSWs of a
 * pair, their monomial factors psi^(e L(j)) - 1 applied slot-wise, one
 * inverse transform per output polynomial; the accumulator is u64. */
static void blind_rotate_torus(or_bsk* K, const uint64_t* ks_lwe, const uint8_t* luts, int n_out, int direct, uint64_t* outs) {
    const or_params* P = &K->P;
    const fft_plan* F = K->FP;
    int k = P->k, N = P->N, n = P->n, M = N / 2, log2N2 = ilog2(2 * N);
    size_t kp1 = (size_t)k + 1, big = (size_t)k * N;
    double* dacc = calloc(kp1 * N, sizeof(double)); /* f64 accumulator (fft.h) */
    uint64_t* acc = calloc(kp1 * N, 8);
    cplx* D = malloc(sizeof(cplx) * kp1 * M);
    cplx* Z = malloc(sizeof(cplx) * M);
    uint64_t* V = malloc(8 * N);
    struct { double cr[3], ci[3]; }* SF = malloc(sizeof(*SF) * M); /* a step's slot factors */
    const uint64_t delta = 1ULL << 59;
    if (direct == 1) {
        int box = N / 16, half = box / 2;
        for (int j = 0; j < N; j++) {
            int m = (j + half) / box;
            V[j] = m < 16 ? (uint64_t)luts[m] * delta : (uint64_t)0 - (uint64_t)luts[0] * delta;
        }
    } else for (int j = 0; j < N; j++) V[j] = delta / 2;
    uint32_t b = mod_switch(ks_lwe[n], log2N2);
    for (int j = 0; j < N; j++) {
        int s = (j + (int)b) & (2 * N - 1);
        dacc[(size_t)k * N + j] = (double)(int64_t)(s < N ? V[s] : (uint64_t)0 - V[s - N]);
    }
    for (int i = 0; i < n; i += 2) {
        uint32_t ai = mod_switch(ks_lwe[i], log2N2);
        uint32_t aj = i + 1 < n ? mod_switch(ks_lwe[i + 1], log2N2) : 0;
        if (ai == 0 && aj == 0) continue;
        for (size_t c = 0; c < kp1; c++) {
            cplx* Dc = D + c * M;
            for (int t = 0; t < M; t++) {
                Dc[t].re = acc_digit(dacc[c * N + t], P->pbs_base_log);
                Dc[t].im = acc_digit(dacc[c * N + t + M], P->pbs_base_log);
            }
            fft_forward(F, Dc);
        }
        /* slot factors: psi^(a_i L), psi^(a_j L) from the quadrant table, and their
         * product for a_i + a_j (N is a power of two: masks and shifts, not divisions) */
        const uint32_t m2N = 2u * (uint32_t)N - 1u, mq = (uint32_t)(N / 2) - 1u;
        const int lq = ilog2(N / 2);
        for (int t = 0; t < M; t++) {
            for (int h = 1; h < 3; h++) {
                uint32_t kk = (uint32_t)((uint64_t)(h == 1 ? ai : aj) * F->leaf[t]) & m2N;
                cplx qv = F->qt[kk & mq];
                quarter_turns(qv.re, qv.im, kk >> lq, &SF[t].cr[h], &SF[t].ci[h]);
            }
            c_mul(SF[t].cr[1], SF[t].ci[1], SF[t].cr[2], SF[t].ci[2], &SF[t].cr[0], &SF[t].ci[0]);
        }
        for (size_t c = 0; c < kp1; c++) {
            for (int t = 0; t < M; t++) {
                const double* cr = SF[t].cr;
                const double* ci = SF[t].ci;
                /* per row r: K_r = sum_g G_g[r][c] (c_g - 1), g ascending; then
                 * z = D_c K_c + sum_(r != c, ascending) D_r K_r (the r = c term first) */
                double kr[8], ki[8]; /* k + 1 <= 8 (or_bsk_prepare) */
                for (size_t r = 0; r < kp1; r++)
                    for (int g = 0; g < 3; g++) {
                        const cplx* G = K->bsk_f + ((size_t)(i / 2) * 3 + g) * kp1 * kp1 * M;
                        const cplx B = G[(r * kp1 + c) * M + t];
                        if (g == 0) c_mul(B.re, B.im, cr[g] - 1.0, ci[g], &kr[r], &ki[r]);
                        else c_mac(B.re, B.im, cr[g] - 1.0, ci[g], &kr[r], &ki[r]);
                    }
                double zr, zi;
                c_mul(D[c * M + t].re, D[c * M + t].im, kr[c], ki[c], &zr, &zi);
                for (size_t r = 0; r < kp1; r++)
                    if (r != c) c_mac(D[r * M + t].re, D[r * M + t].im, kr[r], ki[r], &zr, &zi);
                Z[t].re = zr; Z[t].im = zi;
            }
            fft_inverse(F, Z);
            for (int t = 0; t < M; t++) {
                dacc[c * N + t] = acc_reduce(dacc[c * N + t] + Z[t].re);
                dacc[c * N + t + M] = acc_reduce(dacc[c * N + t + M] + Z[t].im);
            }
        }
    }
    for (size_t c = 0; c < kp1 * (size_t)N; c++) acc[c] = torus_of(dacc[c]);
    int32_t pos[17], d[17];
    for (int f = 0; f < (direct ? 1 : n_out); f++) {
        uint64_t* out = outs + (size_t)f * (big + 1);
        int nt = direct ? 0 : or_lut_terms(N, luts + 16 * f, pos, d);
        for (size_t c = 0; c <= (size_t)k; c++) {
            const uint64_t* A = acc + c * N;
            for (int t = 0; t < (c < (size_t)k ? N : 1); t++) {
                int src0 = t == 0 ? 0 : N - t;
                uint64_t a = 0;
                if (direct) a = A[src0];
                else for (int q = 0; q < nt; q++) {
                    int src = src0 - pos[q];
                    int64_t dd = d[q];
                    if (src < 0) { src += N; dd = -dd; }
                    a += (uint64_t)dd * A[src];
                }
                out[c * N + t] = t == 0 ? a : (uint64_t)0 - a;
            }
        }
        if (direct == 2) out[big] += 1ULL << 58;
    }
    free(acc); free(dacc); free(D); free(Z); free(V); free(SF);
}

void or_blind_rotate_multi(void* pk, const uint64_t* ks_lwe, const uint8_t* luts, int n_out, int direct, uint64_t* outs) {
    or_bsk* K = (or_bsk*)pk;
    if (K->FP) { blind_rotate_torus(K, ks_lwe, luts, n_out, direct, outs); return; }
    const or_params* P = &K->P;
    int k = P->k, N = P->N, n = P->n, log2N2 = ilog2(2 * N);
    size_t kp1 = (size_t)k + 1, big = (size_t)k * N;
    uint64_t* acc = calloc(kp1 * N, 8);
    int64_t* dig = malloc(8 * kp1 * N);
    uint64_t* D = malloc(8 * 2 * kp1 * N);
    uint64_t* res[2] = {malloc(8 * N), malloc(8 * N)};
    uint64_t* V = malloc(8 * N);
    uint64_t* Y = malloc(8 * N);
    /* direct == 1: the LUT polynomial itself; 0 (multi-value) and 2 (sign gate):
     * the constant test polynomial (Delta/2) * sum_j X^j */
    if (direct == 1) make_lut_poly(N, luts, V);
    else for (int j = 0; j < N; j++) V[j] = half_delta_q();
    uint32_t b = mod_switch(ks_lwe[n], log2N2);
    /* acc = (0, X^{-b} V) */
    for (int j = 0; j < N; j++) acc[(size_t)k * N + j] = rot_coef(V, N, j, (2 * N - (int)b) % (2 * N));
    const int U = bsk_unroll(P);
    for (int i = 0; i < n; i += U) {
        /* step over coefficients i .. i+U-1: exponents of the U (or 2^U - 1) terms */
        uint32_t ai = mod_switch(ks_lwe[i], log2N2);
        uint32_t aj = (U == 2 && i + 1 < n) ? mod_switch(ks_lwe[i + 1], log2N2) : 0;
        if (ai == 0 && aj == 0) continue; /* X^0 acc - acc = 0: exactly a no-op */
        uint32_t e[3];
        int nterms = U == 2 ? 3 : 1;
        if (U == 2) { e[0] = (ai + aj) % (2 * (uint32_t)N); e[1] = ai; e[2] = aj; }
        /* signed digits of the decomposed polynomial: (X^a - 1) * acc (plain
         * CMUX) or acc itself (unrolled: the monomials multiply afterwards) */
        for (size_t c = 0; c < kp1; c++) {
            const uint64_t* A = acc + c * N;
            for (int j = 0; j < N; j++)
                dig[c * N + j] = decompose_q(U == 2 ? A[j] : q_sub(rot_coef(A, N, j, (int)ai), A[j]));
        }
        /* NTT of the digit polynomials per prime */
        for (int q = 0; q < 2; q++) {
            const int64_t p = (int64_t)PR[q];
            for (size_t r = 0; r < kp1; r++) {
                uint64_t* Dr = D + (q * kp1 + r) * N;
                for (int j = 0; j < N; j++) Dr[j] = (uint64_t)(((dig[r * N + j] % p) + p) % p);
                nega_forward(K->NP, q, Dr);
            }
        }
        for (int g = 0; g < nterms; g++) {
            if (U == 2 && e[g] == 0) continue; /* (X^0 - 1) * y = 0 */
            const size_t w = U == 2 ? (size_t)(i / 2) * 3 + g : (size_t)i;
            for (size_t c = 0; c < kp1; c++) {
                for (int q = 0; q < 2; q++) {
                    const uint64_t p = PR[q];
                    const uint64_t* Dq = D + q * kp1 * N;
                    const uint64_t* G = K->bsk_ntt[q] + w * kp1 * kp1 * N;
                    for (int t = 0; t < N; t++) {
                        uint64_t s = 0;
                        for (size_t r = 0; r < kp1; r++) s = (s + Dq[r * N + t] * G[(r * kp1 + c) * N + t]) % p;
                        res[q][t] = s;
                    }
                    nega_inverse(K->NP, q, res[q]);
                }
                for (int t = 0; t < N; t++) Y[t] = crt2(res[0][t], res[1][t]);
                /* acc_c += (X^e - 1) * y  (unrolled) or y (plain CMUX) */
                for (int t = 0; t < N; t++) {
                    uint64_t add = U == 2 ? q_sub(rot_coef(Y, N, t, (int)e[g]), Y[t]) : Y[t];
                    acc[c * N + t] = q_add(acc[c * N + t], add);
                }
            }
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
                uint64_t v = t == 0 ? a : q_neg(a);
                out[(size_t)j * N + t] = or_conv(v);
            }
        }
        const uint64_t* B = acc + (size_t)k * N;
        out[big] = or_conv(direct ? B[0] : apply_w(B, N, 0, nt, pos, d));
        if (direct == 2) out[big] += 1ULL << 58; /* sign gate: +-Delta/2 + Delta/2 -> {0, Delta} */
    }
    free(acc); free(dig); free(D); free(res[0]); free(res[1]); free(V); free(Y);
}

/* single LUT, rotating the LUT polynomial itself */
void or_blind_rotate(void* pk, const uint64_t* ks_lwe, const uint8_t lut[16], uint64_t* out) {
    or_blind_rotate_multi(pk, ks_lwe, lut, 1, 1, out);
}

/* ------------------------------------------- exact blind rotation (torus)
 * The torus ring's unrolled CMUX ladder (blind_rotate_torus above) restated in exact
 * integer arithmetic, independently of the f64 FFT's operation sequence: the accumulator
 * is u64 (torus 2^64), the gadget digit of a coefficient is its top 23 bits rounded
 * (signed, |d| <= 2^22, the same rule as acc_digit on the exact value), and every
 * negacyclic product digit x GGSW polynomial is a schoolbook product with wrapping u64
 * arithmetic -- exact mod 2^64.  Per step (pair i, i+1, e = (a_i + a_j, a_i, a_j)):
 *   acc_c += sum_r D_r * H_rc,   H_rc = sum_g (X^e_g - 1) G_g[r][c]
 * which is sum_g (X^e_g - 1) (sum_r D_r G_g[r][c]) by distributivity (exact in Z_2^64[X]).
 * The w-step, sample extraction and sign offset are those of blind_rotate_torus.  Test
 * infrastructure: it pins the f64 ladder (and the device, bit-identical to it) to the exact
 * external products within a stated phase bound (tests/test_exact_br.py). */
/* out += D * H (negacyclic, mod 2^64); D signed with |D| < 2^32 */
static void nega_mac_small(int N, const int64_t* D, const uint64_t* H, uint64_t* out) {
    for (int j = 0; j < N; j++) {
        int64_t d = D[j];
        if (!d) continue;
        const uint64_t m = (uint64_t)(d < 0 ? -d : d); /* < 2^32: two 32 x 32 products per term */
        const int neg = d < 0;
        uint64_t* o = out + j;
        const int n1 = N - j;
        for (int t = 0; t < n1; t++) {
            const uint64_t h = H[t];
            const uint64_t v = m * (uint32_t)h + ((m * (h >> 32)) << 32);
            o[t] += neg ? (uint64_t)0 - v : v;
        }
        o = out - n1; /* X^N = -1: coefficient t + j - N */
        for (int t = n1; t < N; t++) {
            const uint64_t h = H[t];
            const uint64_t v = m * (uint32_t)h + ((m * (h >> 32)) << 32);
            o[t] -= neg ? (uint64_t)0 - v : v;
        }
    }
}
/* (X^e poly)[t], e in [0, 2N), negacyclic, mod 2^64 */
static inline uint64_t rot_u64(const uint64_t* poly, int N, int t, int e) {
    int s = t - e;
    s %= 2 * N; if (s < 0) s += 2 * N;
    return s < N ? poly[s] : (uint64_t)0 - poly[s - N];
}
static void blind_rotate_exact(const or_params* P, const uint64_t* bsk, const uint64_t* ks_lwe, const uint8_t* luts,
                               int n_out, int direct, uint64_t* outs, uint64_t* glwe_out) {
    const int k = P->k, N = P->N, n = P->n, log2N2 = ilog2(2 * N), B = P->pbs_base_log;
    const size_t kp1 = (size_t)k + 1, big = (size_t)k * N;
    uint64_t* acc = calloc(kp1 * N, 8);
    uint64_t* nacc = malloc(8 * kp1 * N);
    int64_t* D = malloc(8 * kp1 * N);
    uint64_t* H = malloc(8 * kp1 * kp1 * N);
    uint64_t* V = malloc(8 * (size_t)N);
    const uint64_t delta = 1ULL << 59;
    if (direct == 1) {
        int box = N / 16, half = box / 2;
        for (int j = 0; j < N; j++) {
            int m = (j + half) / box;
            V[j] = m < 16 ? (uint64_t)luts[m] * delta : (uint64_t)0 - (uint64_t)luts[0] * delta;
        }
    } else for (int j = 0; j < N; j++) V[j] = delta / 2;
    uint32_t b = mod_switch(ks_lwe[n], log2N2);
    for (int j = 0; j < N; j++) acc[(size_t)k * N + j] = rot_u64(V, N, j, (2 * N - (int)b) % (2 * N));
    for (int i = 0; i < n; i += 2) {
        uint32_t ai = mod_switch(ks_lwe[i], log2N2);
        uint32_t aj = i + 1 < n ? mod_switch(ks_lwe[i + 1], log2N2) : 0;
        if (ai == 0 && aj == 0) continue;
        const int e[3] = {(int)((ai + aj) % (2u * (uint32_t)N)), (int)ai, (int)aj};
        /* digits: round(v / 2^(64-B)) of the signed value v (ties away from zero; a tie is an
         * exact half, which the f64 ladder's ties-to-even can only meet on the same value) */
        for (size_t c = 0; c < kp1 * (size_t)N; c++) {
            const int64_t v = (int64_t)acc[c];
            const int sh = 64 - B;
            D[c] = (int64_t)((v >> sh) + ((v >> (sh - 1)) & 1));
        }
        /* H_rc = sum_g (X^e_g - 1) G_g[r][c] */
        for (size_t rc = 0; rc < kp1 * kp1; rc++) {
            uint64_t* h = H + rc * N;
            for (int t = 0; t < N; t++) h[t] = 0;
            for (int g = 0; g < 3; g++) {
                if (e[g] == 0) continue;
                const uint64_t* G = bsk + (((size_t)(i / 2) * 3 + g) * kp1 * kp1 + rc) * N;
                for (int t = 0; t < N; t++) h[t] += rot_u64(G, N, t, e[g]) - G[t];
            }
        }
        memcpy(nacc, acc, 8 * kp1 * N);
        for (size_t c = 0; c < kp1; c++)
            for (size_t r = 0; r < kp1; r++) nega_mac_small(N, D + r * N, H + (r * kp1 + c) * N, nacc + c * N);
        memcpy(acc, nacc, 8 * kp1 * N);
    }
    if (glwe_out) memcpy(glwe_out, acc, 8 * kp1 * N);
    int32_t pos[17], d[17];
    for (int f = 0; f < (direct ? 1 : n_out); f++) {
        uint64_t* out = outs + (size_t)f * (big + 1);
        int nt = direct ? 0 : or_lut_terms(N, luts + 16 * f, pos, d);
        for (size_t c = 0; c <= (size_t)k; c++) {
            const uint64_t* A = acc + c * N;
            for (int t = 0; t < (c < (size_t)k ? N : 1); t++) {
                int src0 = t == 0 ? 0 : N - t;
                uint64_t a = 0;
                if (direct) a = A[src0];
                else for (int q = 0; q < nt; q++) {
                    int src = src0 - pos[q];
                    int64_t dd = d[q];
                    if (src < 0) { src += N; dd = -dd; }
                    a += (uint64_t)dd * A[src];
                }
                out[c * N + t] = t == 0 ? a : (uint64_t)0 - a;
            }
        }
        if (direct == 2) out[big] += 1ULL << 58;
    }
    free(acc); free(nacc); free(D); free(H); free(V);
}
/* count independent exact blind rotations (OpenMP over them): ks_lwe count*(n+1), luts
 * count*n_out*16, outs count*n_out*(kN+1) (direct: n_out = 1) */
void or_blind_rotate_exact(const or_params* P, const uint64_t* bsk, const uint64_t* ks_lwe, const uint8_t* luts,
                           int n_out, int direct, size_t count, uint64_t* outs) {
    const size_t big = (size_t)P->k * P->N, no = direct ? 1 : (size_t)n_out;
    #pragma omp parallel for schedule(dynamic, 1)
    for (long q = 0; q < (long)count; q++)
        blind_rotate_exact(P, bsk, ks_lwe + (size_t)q * (P->n + 1), luts + (size_t)q * no * 16, n_out, direct,
                           outs + (size_t)q * no * (big + 1), NULL);
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
