// ChaCha20 block function (RFC 8439 rounds; key = seed, nonce = stream,
// 64-bit block counter), shared by the host key generator (keys.cpp) and the
// device key generator (keygen.hip), so both draw the same words for the same
// (seed, stream, index).  Word pair (2q, 2q+1) of block b is u64 number 8b + q.
#pragma once
#include <cstdint>

#include "common.h"

namespace fr {

FR_HD uint32_t chacha_rotl(uint32_t a, int b) { return (a << b) | (a >> (32 - b)); }

FR_HD void chacha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d ^= a; d = chacha_rotl(d, 16);
    c += d; b ^= c; b = chacha_rotl(b, 12);
    a += b; d ^= a; d = chacha_rotl(d, 8);
    c += d; b ^= c; b = chacha_rotl(b, 7);
}

FR_HD void chacha_block(uint64_t seed, uint64_t stream, uint64_t counter, uint32_t out[16]) {
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                             (uint32_t)seed, (uint32_t)(seed >> 32), 0x243F6A88u, 0x85A308D3u,
                             0x13198A2Eu, 0x03707344u, 0xA4093822u, 0x299F31D0u,
                             (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream,
                             (uint32_t)(stream >> 32)};
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = in[i];
    for (int i = 0; i < 10; ++i) {
        chacha_qr(x[0], x[4], x[8], x[12]); chacha_qr(x[1], x[5], x[9], x[13]);
        chacha_qr(x[2], x[6], x[10], x[14]); chacha_qr(x[3], x[7], x[11], x[15]);
        chacha_qr(x[0], x[5], x[10], x[15]); chacha_qr(x[1], x[6], x[11], x[12]);
        chacha_qr(x[2], x[7], x[8], x[13]); chacha_qr(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

}  // namespace fr
