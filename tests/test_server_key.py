"""A server that holds only the server key (fr_load_server_key).

Reference: has_match(sk, content, pattern) (src/regex/engine.rs:8) takes the ServerKey
alone; the reference derives it next to the client key in one process (gen_keys,
ciphertext.rs:42-45; ServerKey::new, engine.rs:252).  Here the client exports the server key
(fr_export_server_key) and a server context without any client key installs it.

Pins:
- CPU: export -> load -> export is the identity; wrong lengths are refused; no client key
  is needed (and none appears: serialize_client_key still refuses).
- GPU, every point: /abc/ x 64 encrypted by the client, matched on a server context holding
  only the imported key, decrypts (by the client) to the plaintext oracle's bit, and its
  result words equal those of a context that generated the same key itself.
"""
import numpy as np
import pytest

import fheregex as F
import regex_oracle as ro

SEED = 42


@pytest.fixture(scope="module")
def host_client(key_blob):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(SEED)
    return ctx


def test_load_server_key_roundtrip_host(host_client):
    ksk, bsk = host_client.export_server_key()
    server = F.Context(device=-1)
    server.load_server_key(ksk, bsk)
    k2, b2 = server.export_server_key()
    assert np.array_equal(k2, ksk) and np.array_equal(b2, bsk)
    with pytest.raises(F.FheRegexError):
        server.serialize_client_key()  # the server never saw a client key


def test_server_key_file_roundtrip(host_client, tmp_path):
    """ServerKey.save / ServerKey.load: the arrays through an .npz (no pickle)"""
    path = str(tmp_path / "sk.npz")
    F.ServerKey(host_client).save(path)
    sk = F.ServerKey.load(path, device=-1)
    a, b = host_client.export_server_key()
    a2, b2 = sk.ctx.export_server_key()
    assert np.array_equal(a, a2) and np.array_equal(b, b2)


def test_load_server_key_wrong_lengths(host_client):
    ksk, bsk = host_client.export_server_key()
    server = F.Context(device=-1)
    for k, b in ((ksk[:-1], bsk), (ksk, bsk[:-1]), (ksk, np.zeros(0, np.uint64))):
        with pytest.raises(F.FheRegexError) as e:
            server.load_server_key(k, b)
        assert e.value.code == F.ERR_INVALID
    with pytest.raises(F.FheRegexError):  # nothing was installed
        server.export_server_key()
    # another parameter point's key does not fit this context
    other = F.Context(device=-1, params=F.default_params(k=2, N=1024))
    with pytest.raises(F.FheRegexError):
        other.load_server_key(ksk, bsk)


POINTS = [(F.RING_FFT, 1, 2048), (F.RING_FFT, 2, 1024), (F.RING_RNS, 1, 2048)]


@pytest.mark.gpu
@pytest.mark.parametrize("point", POINTS, ids=["fft", "fft-k2n1024", "rns"])
def test_server_without_client_key(point, key_blob):
    ring, k, N = point
    p = F.default_params(k=k, N=N, ring=ring)
    client = F.Context(device=-1, params=p)  # host: client key, server-key generation, encryption
    client.load_client_key(key_blob)
    client.gen_server_key(SEED)
    ksk, bsk = client.export_server_key()
    server = F.Context(device=0, params=p)  # the server: the imported key only
    server.load_server_key(ksk, bsk)
    both = F.Context(device=0, params=p)  # a context that derives the same key itself
    both.load_client_key(key_blob)
    both.gen_server_key(SEED)
    rng = np.random.default_rng(7)
    for planted in (True, False):
        s = "".join(chr(c) for c in rng.integers(0x20, 0x7F, 64))
        if planted:
            s = s[:30] + "abc" + s[33:]
        exp = ro.has_match(s, "/abc/").result
        ct = client.encrypt_str(s, seed=5)
        out, st = server.has_match(server.upload_radix(ct), "/abc/")
        words = server.download_radix(out)
        assert client.decrypt_radix(words) == exp, (planted, s)
        ref_out, _ = both.has_match(both.upload_radix(ct), "/abc/")
        assert np.array_equal(both.download_radix(ref_out), words)
        assert st.blind_rotations > 0
        # a key installed while a match is still queued (calls are asynchronous): the device
        # drains before the old key's buffers go, and the queued match reads the old key
        queued, _ = server.has_match(server.upload_radix(ct), "/abc/")
        server.load_server_key(ksk, bsk)
        assert np.array_equal(server.download_radix(queued), words)
