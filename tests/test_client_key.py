"""Client-key generation and the bincode client-key writer.

Reference: gen_keys() (src/regex/ciphertext.rs:42-45) calls
gen_keys_radix(&PARAM_MESSAGE_2_CARRY_2, 4) for a fresh RadixClientKey;
generate_test_keys (src/regex/engine.rs:238-246) bincode-serialises one and
read_test_keys (engine.rs:248-254) reads it back.

Pins:
- the writer against the reference's own fixture (test_data/client_key):
  serialize(load(fixture)) is the fixture byte for byte;
- a generated key's parameter block against the fixture's (the reference's
  PARAM_MESSAGE_2_CARRY_2 words, 4 blocks), its layout against the oracle's
  independent parser (oracle_ffi.parse_client_key);
- on the GPU, a whole /abc/ match under a generated key decrypting (by the
  oracle, from the serialised key) to the plaintext oracle's bit.
"""
import numpy as np
import pytest

import fheregex as F
import oracle_ffi as of
import regex_oracle as ro

PARAMS_OFF = 38736  # the parameter block + num_blocks, 17 words


def test_writer_reproduces_fixture(key_blob):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    assert ctx.serialize_client_key() == key_blob


def test_writer_reproduces_fixture_k2n1024(key_blob):
    """the k = 2, N = 1024 context reads the same 2048-bit key; the blob is unchanged"""
    ctx = F.Context(device=-1, params=F.default_params(k=2, N=1024))
    ctx.load_client_key(key_blob)
    assert ctx.serialize_client_key() == key_blob


def test_serialize_without_key():
    ctx = F.Context(device=-1)
    with pytest.raises(F.FheRegexError):
        ctx.serialize_client_key()


@pytest.mark.parametrize("seed", [0, 1, 2**64 - 1])
def test_generated_key_layout(key_blob, seed):
    ctx = F.Context(device=-1)
    ctx.gen_client_key(seed)
    blob = ctx.serialize_client_key()
    assert len(blob) == len(key_blob)
    # the parameter block is the reference's PARAM_MESSAGE_2_CARRY_2, 4 blocks
    assert blob[PARAMS_OFF:] == key_blob[PARAMS_OFF:]
    k = of.parse_client_key(blob)
    assert len(k["s_big"]) == 2048 and len(k["s_small"]) == 742 and k["poly_size"] == 2048
    assert np.array_equal(k["s_big"], k["glwe"])
    for s in (k["s_big"], k["s_small"]):
        assert set(np.unique(s).tolist()) <= {0, 1}
        n = len(s)
        # uniform binary: weight within 6 standard deviations of n/2
        assert abs(int(s.sum()) - n / 2) < 6 * (n / 4) ** 0.5
    # reproducible from the seed; another seed gives another key
    again = F.Context(device=-1)
    again.gen_client_key(seed)
    assert again.serialize_client_key() == blob
    other = F.Context(device=-1)
    other.gen_client_key(seed ^ 0x5A5A)
    assert other.serialize_client_key() != blob


def test_generated_key_roundtrips_through_loader():
    ctx = F.Context(device=-1)
    ctx.gen_client_key(11)
    blob = ctx.serialize_client_key()
    back = F.Context(device=-1)
    back.load_client_key(blob)
    assert back.serialize_client_key() == blob


def test_generated_key_k2n1024_params():
    """at k = 2, N = 1024 the parameter block names that point; the loader takes it"""
    p = F.default_params(k=2, N=1024)
    ctx = F.Context(device=-1, params=p)
    ctx.gen_client_key(5)
    blob = ctx.serialize_client_key()
    k = of.parse_client_key(blob)
    assert (k["k"], k["N"], k["poly_size"], len(k["s_big"])) == (2, 1024, 1024, 2048)
    back = F.Context(device=-1, params=p)
    back.load_client_key(blob)
    assert back.serialize_client_key() == blob


def test_generated_key_encrypts_and_decrypts():
    """encrypt_str under a generated key decrypts with the oracle's reading of the
    serialised key (an independent decryption), and the host server key derived from
    it equals the oracle's keygen word for word"""
    ctx = F.Context(device=-1)
    ctx.gen_client_key(99)
    key = of.parse_client_key(ctx.serialize_client_key())
    O = of.Oracle(key, seed=3, with_bsk=False)
    ct = ctx.encrypt_str("Hi, regex!", seed=4)
    for i, ch in enumerate(b"Hi, regex!"):
        assert O.decrypt_radix(ct[i]) == ch
        assert ctx.decrypt_radix(ct[i]) == ch
    # the keyswitching key of ServerKey::new (engine.rs:252) under this key
    ctx.set_keygen(F.KEYGEN_HOST)
    ctx.gen_server_key(3)
    ksk, _ = ctx.export_server_key()
    assert np.array_equal(ksk, O.ksk)
    # a keyswitched block decrypts under the generated small key
    ks = O.keyswitch(ct[0][0])
    ph = int((int(ks[0][-1]) - int(np.dot(ks[0][:-1], key["s_small"]).astype(np.uint64))) % 2**64)
    assert of.lib().or_decode16(ph) == ord("H") & 3


def test_gen_keys_without_blob_host():
    """fheregex.gen_keys() with no blob, as the reference's gen_keys() (ciphertext.rs:42-45)"""
    ck, sk = F.gen_keys(device=-1, client_seed=8)
    blob = ck.serialize()
    assert len(blob) == 38872
    ck2, _ = F.gen_keys(device=-1, client_seed=8)
    assert ck2.serialize() == blob
    h = ck.ctx.encrypt_str("abc", seed=1)
    assert [ck.ctx.decrypt_radix(h[i]) for i in range(3)] == [97, 98, 99]


def test_c_abi_symbols_declared():
    hdr = open(F.HEADER).read()
    for sym in ("fr_gen_client_key", "fr_serialize_client_key"):
        assert sym + "(" in hdr
        assert hasattr(F.lib(), sym)


@pytest.mark.gpu
@pytest.mark.parametrize("kN", [(1, 2048), (2, 1024)], ids=["fft", "fft-k2n1024"])
def test_match_under_generated_key(kN):
    """/abc/ x 64 end to end under a freshly generated key: the device encrypts, keys and
    matches; the oracle decrypts the result from the serialised key and one bootstrap is
    bit-exact against the oracle's keys derived from that key"""
    k, N = kN
    ck, sk = F.gen_keys(device=0, params=F.default_params(k=k, N=N), seed=42, client_seed=2024)
    ctx = ck.ctx
    key = of.parse_client_key(ck.serialize())
    rng = np.random.default_rng(64)
    for planted in (True, False):
        s = "".join(chr(c) for c in rng.integers(0x20, 0x7F, 64))
        if planted:
            s = s[:17] + "abc" + s[20:]
        exp = ro.has_match(s, "/abc/")
        hs = ctx.encrypt_upload_str(s, seed=7)
        out = F.has_match(sk, hs, "/abc/")
        blocks = ctx.download_radix(out)
        O = of.Oracle(key, seed=42, k=k, N=N, with_bsk=False)
        assert O.decrypt_radix(blocks) == exp.result == ck.decrypt(out), (planted, s)
    O = of.Oracle(key, seed=42, k=k, N=N)
    ks = O.keyswitch(O.encrypt_blocks([6], seed=3))
    lut = [(5 * m + 1) % 16 for m in range(16)]
    dev = ctx.dev_blind_rotate(ks, [lut])[0]
    assert (dev == O.blind_rotate(ks[0], lut)).all()
    assert int(O.decode16(dev)[0]) == lut[6]


@pytest.mark.gpu
@pytest.mark.parametrize("kN", [(1, 2048), (2, 1024)], ids=["fft", "fft-k2n1024"])
def test_device_keygen_and_encryption_under_generated_key(kN):
    """ServerKey::new (engine.rs:252) on the device under a freshly generated client key gives
    the host generator's key word for word, and encrypt_str on the device (ciphertext.rs:32-40)
    the host encryption's words, as with the fixture key (tests/test_keygen.py,
    tests/test_client.py)"""
    k, N = kN
    p = F.default_params(k=k, N=N)
    dev = F.Context(device=0, params=p)
    dev.gen_client_key(77)
    dev.set_keygen(F.KEYGEN_DEVICE)
    dev.gen_server_key(5)
    host = F.Context(device=-1, params=p)
    host.load_client_key(dev.serialize_client_key())
    host.gen_server_key(5)
    dk, db = dev.export_server_key()
    hk, hb = host.export_server_key()
    assert np.array_equal(dk, hk) and np.array_equal(db, hb)
    s = "GPU-encrypted, generated key"
    hs = dev.encrypt_upload_str(s, seed=9)
    ref = host.encrypt_str(s, seed=9)
    for i in range(len(s)):
        assert np.array_equal(dev.download_radix(hs[i]), ref[i]), i
        assert dev.decrypt_radix(ref[i]) == ord(s[i])
