"""Server-key generation on the device (ServerKey::new at
src/regex/engine.rs:252).  The device generator must give the host
generator's key word for word, and the host generator is pinned to the
oracle's keygen (tests/test_fft.py::test_torus_server_key_matches_oracle).
Every bit-exact blind-rotation test in test_gpu.py / test_fft.py also runs on
a device-generated key (gctx uses KEYGEN_AUTO), which covers the on-device
Fourier transform of the BSK."""
import time

import numpy as np
import pytest

import fheregex as F

SEED = 42


def test_keygen_setting_host_only(key_blob):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    ctx.set_keygen(F.KEYGEN_HOST)
    ctx.set_keygen(F.KEYGEN_AUTO)
    with pytest.raises(F.FheRegexError):
        ctx.set_keygen(3)
    ctx.set_keygen(F.KEYGEN_DEVICE)
    with pytest.raises(F.FheRegexError):
        ctx.gen_server_key(SEED)  # no device


@pytest.fixture(scope="module")
def host_keys(key_blob):
    ctx = F.Context(device=-1)
    ctx.load_client_key(key_blob)
    ctx.gen_server_key(SEED)
    return ctx.export_server_key()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [SEED, 7])
def test_device_keygen_matches_host(key_blob, seed, host_keys):
    ctx = F.Context(device=0)
    ctx.load_client_key(key_blob)
    ctx.set_keygen(F.KEYGEN_DEVICE)
    t0 = time.perf_counter()
    ctx.gen_server_key(seed)
    dt = time.perf_counter() - t0
    ksk, bsk = ctx.export_server_key()
    if seed == SEED:
        hk, hb = host_keys
    else:
        h = F.Context(device=-1)
        h.load_client_key(key_blob)
        h.gen_server_key(seed)
        hk, hb = h.export_server_key()
    assert np.array_equal(ksk, hk)
    assert np.array_equal(bsk, hb)
    print(f"device keygen {dt * 1e3:.1f} ms")


@pytest.mark.gpu
def test_device_key_runs_bit_exact(key_blob):
    """A device-generated key and a host-generated (uploaded) key give the
    same bootstrapped ciphertexts."""
    outs = []
    for where in (F.KEYGEN_DEVICE, F.KEYGEN_HOST):
        ctx = F.Context(device=0)
        ctx.load_client_key(key_blob)
        ctx.set_keygen(where)
        ctx.gen_server_key(SEED)
        hs = ctx.upload_radix(ctx.encrypt_str("xyabcz", seed=3))
        out, _ = ctx.has_match(hs, "/abc/")
        outs.append(ctx.download_radix(out))
        assert ctx.decrypt_radix(outs[-1]) == 1
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
def test_device_keygen_k2n1024_matches_host(key_blob):
    """BASELINE's "N = 1024" point (k = 2, N = 1024, FFT ring): k_gen_bsk<1024>
    and k_bsk_fourier<1024> against the host generator, then one match."""
    params = F.default_params(k=2, N=1024, ring=F.RING_FFT)
    keys = []
    for where in (F.KEYGEN_DEVICE, F.KEYGEN_HOST):
        ctx = F.Context(device=0 if where == F.KEYGEN_DEVICE else -1, params=params)
        ctx.load_client_key(key_blob)
        ctx.set_keygen(where)
        ctx.gen_server_key(SEED)
        keys.append(ctx.export_server_key())
        if where == F.KEYGEN_DEVICE:
            hs = ctx.upload_radix(ctx.encrypt_str("zabcz", seed=3))
            out, _ = ctx.has_match(hs, "/abc/")
            assert ctx.decrypt_radix(ctx.download_radix(out)) == 1
    assert np.array_equal(keys[0][0], keys[1][0])
    assert np.array_equal(keys[0][1], keys[1][1])
