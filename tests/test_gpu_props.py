"""Randomised parity properties of the GPU codec vs the oracle (hypothesis,
derandomised so every run draws the same cases).

For random (k, m, shard length, erasure set) — m = 0 and k + m = 256
included — through the klauspost-shaped host API (include/hbec.h):
  * Encode == oracle parity (bit-exact),
  * Reconstruct restores every erased shard, ReconstructData every erased
    data shard and nothing else,
  * Verify is true on the codeword and false after any single-byte flip,
  * encode is linear: parity(a ^ b) == parity(a) ^ parity(b).
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu

_codecs = {}


def codec(k, m):
    if (k, m) not in _codecs:
        _codecs[(k, m)] = (RS.New(k, m), CO.build_matrix(k, m))
    return _codecs[(k, m)]


@st.composite
def cases(draw):
    k = draw(st.integers(1, 24))
    m = draw(st.integers(0, 8))
    n = draw(st.sampled_from([1, 2, 15, 16, 17, 63, 64, 1000, 1024, 4095, 4096, 4097, 65536, 70001]))
    seed = draw(st.integers(0, 2**31 - 1))
    n_miss = draw(st.integers(0, m))
    miss = draw(st.lists(st.integers(0, k + m - 1), min_size=n_miss, max_size=n_miss, unique=True))
    return k, m, n, seed, sorted(miss)


SETTINGS = settings(max_examples=120, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])


@SETTINGS
@given(cases())
def test_random_codewords(case):
    k, m, n, seed, miss = case
    enc, mat = codec(k, m)
    rng = np.random.default_rng(seed)
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    shards = [d.copy() for d in data] + [np.zeros(n, np.uint8) for _ in range(m)]
    enc.Encode(shards)
    if m:
        want = CO.apply(mat[k:], data)
        for r in range(m):
            assert np.array_equal(shards[k + r], want[r])
    assert enc.Verify(shards)
    orig = [s.copy() for s in shards]
    if m:
        flip = int(rng.integers(0, k + m))
        pos = int(rng.integers(0, n))
        shards[flip][pos] ^= 1 + int(rng.integers(0, 255))
        assert not enc.Verify(shards)
        shards[flip][:] = orig[flip]
    # Reconstruct: every erased shard comes back
    work = [s.copy() for s in orig]
    for i in miss:
        work[i] = np.zeros(0, np.uint8)
    enc.Reconstruct(work)
    for i in range(k + m):
        assert np.array_equal(work[i], orig[i]), (k, m, n, miss, i)
    # ReconstructData: erased data shards back, erased parity left empty
    work = [s.copy() for s in orig]
    for i in miss:
        work[i] = np.zeros(0, np.uint8)
    enc.ReconstructData(work)
    for i in range(k + m):
        if i < k or i not in miss:
            assert np.array_equal(work[i], orig[i])
        else:
            assert work[i].size == 0


@SETTINGS
@given(st.integers(1, 16), st.integers(1, 6), st.sampled_from([16, 1000, 4096, 65536]), st.integers(0, 2**31 - 1))
def test_encode_is_linear(k, m, n, seed):
    enc, _ = codec(k, m)
    rng = np.random.default_rng(seed)
    a = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    b = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    sa = a + [np.zeros(n, np.uint8) for _ in range(m)]
    sb = b + [np.zeros(n, np.uint8) for _ in range(m)]
    sab = [x ^ y for x, y in zip(a, b)] + [np.zeros(n, np.uint8) for _ in range(m)]
    for s in (sa, sb, sab):
        enc.Encode(s)
    for r in range(m):
        assert np.array_equal(sab[k + r], sa[k + r] ^ sb[k + r])


@pytest.mark.parametrize("k,m", [(128, 128), (255, 1), (1, 255), (200, 56), (17, 0)])
def test_maximum_shard_counts(k, m):
    enc, mat = codec(k, m)
    n = 4096 + 48
    rng = np.random.default_rng(k * 1000 + m)
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    shards = [d.copy() for d in data] + [np.zeros(n, np.uint8) for _ in range(m)]
    enc.Encode(shards)
    if m:
        want = CO.apply(mat[k:], data)
        for r in range(m):
            assert np.array_equal(shards[k + r], want[r])
    # lose the first min(m, k) data shards (all survivors drawn from parity where possible)
    lost = list(range(min(m, k)))
    orig = [s.copy() for s in shards]
    for i in lost:
        shards[i] = np.zeros(0, np.uint8)
    enc.Reconstruct(shards)
    for i in range(k + m):
        assert np.array_equal(shards[i], orig[i])
