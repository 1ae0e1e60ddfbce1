// Host side of the f64 negacyclic FFT (fft.h): twiddle tables and the
// one-time transform of the bootstrapping key into the Fourier domain.
#include "fft.h"

#include <thread>

namespace fr {
namespace fft {

c64 psi_pow(int N, int64_t x) {
    const int64_t twoN = 2 * (int64_t)N, quarter = N / 2;
    x %= twoN;
    if (x < 0) x += twoN;
    const uint32_t q = (uint32_t)(x / quarter);
    const int64_t r = x % quarter;
    const double ang = (double)r * (3.14159265358979323846 / (double)N);
    c64 z;
    psi_quadrant(std::cos(ang), std::sin(ang), q, z.re, z.im);
    return z;
}

Tables::Tables(int n) : N(n), M(n / 2) {
    while ((1 << LOG) < M) ++LOG;
    if ((1 << LOG) != M || N < 8) throw Error(FR_ERR_INVALID, "fft: N must be a power of two >= 8");
    tw.assign(M, c64{0, 0});
    qt.resize(N / 2);
    leaf.resize(M);
    for (int r = 0; r < N / 2; ++r) qt[r] = psi_pow(N, r);
    // exponents of the split tree, level by level
    std::vector<int64_t> E(1, M), next;
    for (int s = 0; s < LOG; ++s) {
        next.assign((size_t)2 << s, 0);
        for (int b = 0; b < (1 << s); ++b) {
            const int64_t e = E[b];
            if (e % 2) throw Error(FR_ERR_INVALID, "fft: odd split exponent");
            tw[(1 << s) + b] = psi_pow(N, e / 2);
            next[2 * b] = (e / 2) % (2 * N);
            next[2 * b + 1] = (e / 2 + N) % (2 * N);
        }
        E.swap(next);
    }
    for (int j = 0; j < M; ++j) leaf[j] = (uint16_t)E[j];
    // the radix-4 forms (fft_br.hip, inv_r4) take a stage's odd sibling as i times the
    // even one: psi^(x + N/2) = i psi^x is an exact quarter turn of psi_pow
    for (int s = 1; s < LOG; ++s)
        for (int b = 0; b < (1 << (s - 1)); ++b) {
            const c64 u = tw[(1 << s) + 2 * b], v = tw[(1 << s) + 2 * b + 1];
            if (v.re != -u.im || v.im != u.re) throw Error(FR_ERR_INVALID, "fft: sibling twiddles are not i apart");
        }
}

void Tables::forward(c64* z) const {
    for (int s = 0; s < LOG; ++s) {
        const int h = M >> (s + 1);
        for (int b = 0; b < (1 << s); ++b) {
            const c64 c = tw[(1 << s) + b];
            for (int j = b * 2 * h; j < b * 2 * h + h; ++j) fwd_bf(z[j].re, z[j].im, z[j + h].re, z[j + h].im, c.re, c.im);
        }
    }
}

void Tables::inverse(c64* z) const {
    if (LOG % 2 == 0) {  // stages (2p + 1, 2p) as radix-4 groups (inv_r4)
        for (int s0 = LOG - 2; s0 >= 0; s0 -= 2) {
            const int s1 = s0 + 1, h1 = M >> (s1 + 1), h0 = 2 * h1;
            for (int b = 0; b < (1 << s0); ++b) {
                const c64 c = tw[(1 << s0) + b], ca = tw[(1 << s1) + 2 * b];
                c64 cc;
                cmul(c.re, c.im, ca.re, ca.im, cc.re, cc.im);
                for (int j = b * 2 * h0; j < b * 2 * h0 + h1; ++j)
                    inv_r4(z[j].re, z[j].im, z[j + h1].re, z[j + h1].im, z[j + h0].re, z[j + h0].im, z[j + h0 + h1].re,
                           z[j + h0 + h1].im, c.re, c.im, ca.re, ca.im, cc.re, cc.im);
            }
        }
        return;
    }
    for (int s = LOG - 1; s >= 0; --s) {
        const int h = M >> (s + 1);
        for (int b = 0; b < (1 << s); ++b) {
            const c64 c = tw[(1 << s) + b];
            for (int j = b * 2 * h; j < b * 2 * h + h; ++j) inv_bf(z[j].re, z[j].im, z[j + h].re, z[j + h].im, c.re, c.im);
        }
    }
}

void bsk_to_fourier(const Tables& T, const std::vector<uint64_t>& bsk, size_t polys, std::vector<c64>& out) {
    const int N = T.N, M = T.M;
    if (bsk.size() != polys * (size_t)N) throw Error(FR_ERR_INVALID, "bsk_to_fourier: size");
    out.resize(polys * (size_t)M);
    const double scale = fourier_key_scale(T.LOG);  // 1/M and the accumulator unit (fft.h), exact
    unsigned hw = std::thread::hardware_concurrency();
    const size_t nt = hw ? (hw > 16 ? 16 : hw) : 4;
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (size_t p = t; p < polys; p += nt) {
                const uint64_t* a = bsk.data() + p * N;
                c64* z = out.data() + p * M;
                for (int k = 0; k < M; ++k) z[k] = c64{(double)(int64_t)a[k], (double)(int64_t)a[k + M]};
                T.forward(z);
                for (int k = 0; k < M; ++k) {
                    z[k].re *= scale;
                    z[k].im *= scale;
                }
            }
        });
    for (auto& x : th) x.join();
}

}  // namespace fft
}  // namespace fr
