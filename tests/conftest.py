import os
import sys

import pytest
# torch first: its wheel bundles its own HIP runtime (libamdhip64, same soname as
# /opt/rocm's); loaded after libfheregex.so's, torch would find no device.  With torch's
# loaded first, libfheregex.so binds to that one runtime (as in bench.py).
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "fhe-regex_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device 0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


# tests/test_gpu.py's RNS point: word-for-word whole-match comparisons whose oracle side
# (the CPU RNS ring) takes 10-100 s each; run with FR_TEST_RNS=1 (the full matrix,
# profiles/r06/gpu_tests_rns_matrix.log), deselected (not skipped) otherwise
RNS_HEAVY = {"test_match_words_fuzz_scale", "test_match_words_full_size_configs", "test_faithful_tree_fuzz_scale",
             "test_faithful_tree_full_metric", "test_match_words_lowering_variants", "test_match_words_start_shards",
             "test_match_parts_words_start_shards"}


def pytest_collection_modifyitems(config, items):
    if os.environ.get("FR_TEST_RNS") == "1":
        return
    keep, drop = [], []
    for it in items:
        cs = getattr(it, "callspec", None)
        heavy = it.originalname in RNS_HEAVY if hasattr(it, "originalname") else False
        if heavy and cs is not None and "rns" in cs.id.split("-"):
            drop.append(it)
        else:
            keep.append(it)
    if drop:
        config.hook.pytest_deselected(items=drop)
        items[:] = keep


@pytest.fixture(scope="session")
def key_blob():
    with open(os.path.join(GOLDEN, "client_key"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def fixture_key():
    import oracle_ffi
    return oracle_ffi.load_fixture_key(os.path.join(GOLDEN, "client_key"))


@pytest.fixture(scope="session")
def oracle_k1(fixture_key):
    """Oracle keys (k=1, N=2048, default ring: the f64-FFT torus) for server-key seed 42."""
    import oracle_ffi
    return oracle_ffi.Oracle(fixture_key, seed=42)


@pytest.fixture(scope="session")
def oracle_rns(fixture_key):
    """Oracle keys on the RNS ring (Z_Q, two-prime NTT), k=1, N=2048, seed 42."""
    import oracle_ffi
    return oracle_ffi.Oracle(fixture_key, seed=42, ring=oracle_ffi.RING_RNS)
