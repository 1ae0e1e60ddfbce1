"""Client side at scale: encrypt_str on the device
(src/regex/ciphertext.rs:32-40) and the bincode RadixCiphertext wire format.
The device encryption must give fr_encrypt_str's words exactly (host
restatement, pinned to the oracle in test_oracle.py).  The wire layout follows
the verified client-key conventions; its agreement with tfhe-rs is [ext]
unverified (tfhe-rs is absent)."""
import struct

import numpy as np
import pytest

import fheregex as F


@pytest.fixture(scope="module")
def hctx(key_blob):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    return ctx


def test_wire_roundtrip(hctx):
    ct = hctx.encrypt_str("hi!", seed=9)
    for ch in range(3):
        data = hctx.serialize_radix(ct[ch])
        L = hctx.lwe_len
        assert len(data) == 8 + 4 * 8 * (L + 4)
        assert struct.unpack_from("<Q", data, 0)[0] == 4
        assert struct.unpack_from("<Q", data, 8)[0] == L
        deg, mm, cm = struct.unpack_from("<QQQ", data, 16 + 8 * L)
        assert (deg, mm, cm) == (3, 4, 4)
        back = hctx.deserialize_radix(data)
        assert np.array_equal(back, ct[ch])
        assert hctx.decrypt_radix(back) == ord("hi!"[ch])


def test_wire_rejects_malformed(hctx):
    data = hctx.serialize_radix(hctx.encrypt_str("a", seed=1)[0])
    with pytest.raises(F.FheRegexError):
        hctx.deserialize_radix(data[:-1])
    with pytest.raises(F.FheRegexError):
        hctx.deserialize_radix(data + b"\0")
    bad = bytearray(data)
    struct.pack_into("<Q", bad, 8, 2048)  # LWE size of another parameter set
    with pytest.raises(F.FheRegexError):
        hctx.deserialize_radix(bytes(bad))
    bad = bytearray(data)
    struct.pack_into("<Q", bad, 16 + 8 * hctx.lwe_len + 8, 8)  # message modulus
    with pytest.raises(F.FheRegexError):
        hctx.deserialize_radix(bytes(bad))
    bad = bytearray(data)
    struct.pack_into("<Q", bad, 0, 1 << 40)
    with pytest.raises(F.FheRegexError):
        hctx.deserialize_radix(bytes(bad))
    # a block with carries (degree > message_modulus - 1) is refused, not decoded wrong
    bad = bytearray(data)
    struct.pack_into("<Q", bad, 16 + 8 * hctx.lwe_len, 4)
    with pytest.raises(F.FheRegexError, match="degree"):
        hctx.deserialize_radix(bytes(bad))
    assert hctx.serialize_radix(hctx.encrypt_str("a", seed=1)[0], degree=3)  # clean blocks still accepted


def test_device_encryption_needs_device(hctx):
    with pytest.raises(F.FheRegexError):
        hctx.encrypt_upload_str("abc", seed=1)


@pytest.mark.gpu
def test_device_encryption_matches_host(key_blob):
    ctx = F.Context(device=0)
    ctx.load_client_key(key_blob)
    rng = np.random.default_rng(4)
    s = "".join(chr(c) for c in rng.integers(0x20, 0x7F, 256))
    hs = ctx.encrypt_upload_str(s, seed=77)
    ref = ctx.encrypt_str(s, seed=77)
    for i in (0, 1, 128, 255):
        assert np.array_equal(ctx.download_radix(hs[i]), ref[i]), i
    got = np.stack([ctx.download_radix(h) for h in hs]).reshape(ref.shape)
    assert np.array_equal(got, ref)
    with pytest.raises(ValueError):  # FR_ERR_NON_ASCII, like the reference's encrypt_str
        ctx.encrypt_upload_str("caf\xe9", seed=1)


@pytest.mark.gpu
def test_device_encrypted_content_matches(key_blob):
    ctx = F.Context(device=0)
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(42)
    hs = ctx.encrypt_upload_str("xx abc yy", seed=5)
    out, _ = ctx.has_match(hs, "/abc/")
    data = ctx.serialize_radix(ctx.download_radix(out))
    assert ctx.decrypt_radix(ctx.deserialize_radix(data)) == 1
