// Client key (reference fixture layout), deterministic server-key generation,
// client-side encryption — host C++.
#pragma once
#include <cstdint>
#include <vector>

#include "common.h"

namespace fr {

// ChaCha20 (DJB layout: 64-bit block counter, 64-bit stream id); key words =
// seed (2 words) + 6 fixed constants.  u64 number idx of a stream is words
// 2*(idx%8), 2*(idx%8)+1 of block idx/8 — random access, so keygen is
// parallel and deterministic.
enum Stream : uint64_t {
    STREAM_KSK_MASK = 1,
    STREAM_KSK_NOISE = 2,
    STREAM_BSK_MASK = 3,
    STREAM_BSK_NOISE = 4,
    STREAM_ENC_MASK = 5,
    STREAM_ENC_NOISE = 6,
    STREAM_CLIENT_KEY = 7,
};

class Rng {
  public:
    Rng(uint64_t seed, uint64_t stream) : seed_(seed), stream_(stream) {}
    uint64_t u64(uint64_t idx);
    // Box-Muller on words 2*idx, 2*idx+1; z * sigma * scale rounded to an
    // integer (scale 2^64: torus units; scale Q: units of Z_Q).
    int64_t gaussian(uint64_t idx, double sigma, double scale = 18446744073709551616.0);

  private:
    uint64_t seed_, stream_, blk_ = 0;
    bool valid_ = false;
    uint32_t w_[16];
};

struct ClientKey {
    std::vector<uint64_t> s_big;    // flattened GLWE key (2048 bits)
    std::vector<uint64_t> s_small;  // LWE key after keyswitch (742 bits)
    int n = 0, k = 0, N = 0;
    int pbs_base_log = 0, pbs_level = 0, ks_base_log = 0, ks_level = 0;
    double lwe_sigma = 0, glwe_sigma = 0;
    uint64_t message_modulus = 0, carry_modulus = 0, num_blocks = 0;
    // the remaining words of the bincode layout, kept as read so that
    // serialize_client_key(parse_client_key(b)) == b: the GLWE key's own data
    // (equal to s_big in every tfhe-rs key) and polynomial_size, and the 17 words
    // of the parameter block + num_blocks (offsets 38736..38871)
    std::vector<uint64_t> s_glwe;
    uint64_t glwe_poly_size = 0;
    uint64_t raw_params[17] = {};
};

// Parse the bincode RadixClientKey of the reference fixture.
ClientKey parse_client_key(const uint8_t* data, size_t len);
// The same layout written back (engine.rs:238-246 generate_test_keys: bincode::serialize
// of the RadixClientKey); byte-identical to the blob a key was parsed from.
std::vector<uint8_t> serialize_client_key(const ClientKey& ck);
// A fresh RadixClientKey (gen_keys_radix(&PARAM_MESSAGE_2_CARRY_2, 4), ciphertext.rs:42-45):
// uniform binary GLWE key of k*N bits (its flattening is the big LWE key) and uniform binary
// LWE key of n bits, from a ChaCha20 stream of `seed` (STREAM_CLIENT_KEY); parameter block
// from p (PARAM_MESSAGE_2_CARRY_2's words at the default params: pfks = (1, 2^23, glwe
// sigma), cbs = (0, 0), message and carry modulus 4, 4 blocks).
ClientKey gen_client_key(const Params& p, uint64_t seed);

// KSK: [i in kN][level j][t in n+1], torus 2^64.
void gen_ksk(const Params& p, const ClientKey& ck, uint64_t seed, std::vector<uint64_t>& ksk);
// BSK: [GGSW w][row r in k+1][component c in k+1][coef], coefficient domain mod Q (rns.h);
// GGSW w per Params::bsk_unroll (k = 1: 3 per pair of LWE coefficients).
void gen_bsk(const Params& p, const ClientKey& ck, uint64_t seed, std::vector<uint64_t>& bsk);
// Host parts of the device key generator (Device::gen_server_key): the
// Box-Muller noise of every KSK row (lwe sigma, torus units), of every BSK
// body coefficient ([w][r][coef], glwe sigma, torus units) and the message bit
// of every GGSW.
void gen_ksk_noise(const Params& p, uint64_t seed, std::vector<int64_t>& e);
void gen_bsk_noise_torus(const Params& p, uint64_t seed, std::vector<int32_t>& e);
std::vector<uint8_t> ggsw_messages(const Params& p, const ClientKey& ck);
// noise of encrypt_blocks for blocks first_block .. first_block + count - 1
void enc_noise(const Params& p, uint64_t seed, uint64_t first_block, size_t count, std::vector<int64_t>& e);

// Fresh LWE encryptions of block messages (Delta = 2^59) under the big key.
void encrypt_blocks(const Params& p, const ClientKey& ck, const uint8_t* msgs, size_t count, uint64_t seed,
                    uint64_t first_block, uint64_t* out /* count * (kN+1) */);
uint64_t lwe_phase(const Params& p, const ClientKey& ck, const uint64_t* lwe);
// tfhe-rs shortint decrypt_message_and_carry: round(phase / Delta) mod 16
uint32_t decode16(uint64_t phase);

// Host negacyclic NTT over Z_p for the two RNS primes (merged-psi
// Cooley-Tukey / Gentleman-Sande, bit-reversed evaluation order) — used by
// keygen and for the device twiddles.  Canonical residues, plain '%' math.
struct NttTables {
    int N = 0, logN = 0;
    std::vector<uint32_t> zeta[2], izeta[2];  // zeta[k] = psi^brv(k), izeta[k] = psi^-brv(k)
    uint32_t n_inv[2] = {0, 0};
    explicit NttTables(int N);
    void forward(int q, uint32_t* a) const;
    void inverse(int q, uint32_t* a) const;  // includes the 1/N factor
};
// negacyclic product mod Q of a, b in [0, Q)
void ring_mul_q(const NttTables& T, const uint64_t* a, const uint64_t* b, uint64_t* out);

}  // namespace fr
