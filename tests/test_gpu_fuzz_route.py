"""Seeded fuzz over the kernel routes of apply_views and Verify: random
(k, m), shard lengths on and off the 16-B and 128-B grids and either side of
the record-kernel thresholds (csrc/hbec.cpp rec_route, tuning.h), random base
offsets and object pitches, random erasure sets.  Every parity byte, every
rebuilt shard and every Verify flag is checked against the oracle
(reedsolomon.New / Encode / Reconstruct semantics, objectserver/ecutils.go:
27,59,111), so whichever kernel a case lands on — packed, pipelined,
streaming, gf_odd, gf_odd_rec tables or bit-plane, gf_wide — it must agree.
"""
import os

import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

import route_rule as R

pytestmark = pytest.mark.gpu

_S_CHOICES = [R.MIN_S_BIG - 16, R.MIN_S_BIG, R.MIN_S - 16, R.MIN_S, R.MIN_S + 16, R.MIN_S + 128, R.MIN_S + 1,
              R.MIN_S + 8, 65536, 65536 + 16, 98304 + 80, 3072, 4096 + 16, 24576 + 128,
              # round 6: the packed limit of 5 <= k <= 8 (32 KiB), odd mid-size shards (fused guard
              # band), and either side of one and two tiles per shard (992-B and 2016-B tiles:
              # the guard band is fused from two tiles up)
              32768, 32784, 4095, 8191, 16383, 161, 1087, 1088, 1089, 2111, 2112, 2113]


def _case(seed):
    rng = np.random.default_rng(0x5EED0000 + seed)
    k = int(rng.integers(2, 13))
    m = int(rng.integers(1, 5))
    s = int(rng.choice(_S_CHOICES))
    off = int(rng.choice([0, 16, 48, 128, 3]))
    pad = int(rng.choice([0, 16, 128, 5]))
    return k, m, s, off, pad, rng


# HBEC_FUZZ_SEEDS widens a one-off run (2000 seeds: profiles/r05_gpu_fuzz_route.txt)
@pytest.mark.parametrize("seed", range(int(os.environ.get("HBEC_FUZZ_SEEDS", "96"))))
def test_fuzz_routes_against_oracle(seed):
    k, m, s, off, pad, rng = _case(seed)
    n = max(2, min(12, 2_500_000 // ((k + m) * s)))
    pitch = (k + m) * s + pad
    buf = torch.empty(off + n * pitch + 64, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(buf.view(1, -1), buf.numel(), first=seed)
    views = [(buf.data_ptr() + off + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = off + o * pitch
        want = CO.apply(rows, [got[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[b + (k + r) * s:b + (k + r + 1) * s], want[r]), (k, m, s, off, pad, o, r)
    # a random erasure set of up to m shards, rebuilt in place
    lost = sorted(rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False).tolist())
    ref = buf.clone()
    for o in range(n):
        for i in lost:
            a = off + o * pitch + i * s
            buf[a:a + s] = 0x6B
    B.reconstruct_views(enc, views, [0 if i in lost else 1 for i in range(k + m)], n, s)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref), (k, m, s, off, pad, lost)
    # Verify: clean, then one flipped byte in one object
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0
    o, i, p = int(rng.integers(0, n)), int(rng.integers(0, k + m)), int(rng.integers(0, s))
    buf[off + o * pitch + i * s + p] ^= 0x80
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == [o], (k, m, s, off, pad, o, i, p)
