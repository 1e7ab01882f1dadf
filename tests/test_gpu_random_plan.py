"""The nursery batch shape: one object plan of objects of
arbitrary, widely spread sizes, every parity byte against the oracle.

A nursery scan hands the stabilizer the oldest objects of a device whatever
their sizes (objectserver/indexdb.go:26,548-557, ecengine.go:583-640), so
S = ceil(len / k) (ecutils.go:14-24) takes hundreds of values in one batch.
Plans code them from per-stripe records over a tile list (plan.cpp
build_tile_lists, odd_impl.h gf_odd_rec LIST): one launch per pass, no size
classes.  Also a Reconstruct of random erasures on the same plan.
"""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,m,n,lo,hi", [(4, 2, 1024, 4096, 1 << 20), (8, 3, 1024, 4096, 1 << 20),
                                         (10, 4, 512, 4096, 1 << 20), (12, 4, 256, 17, 1 << 19),
                                         (6, 3, 512, 17, 300_000), (16, 4, 96, 4096, 1 << 19)])
def test_random_size_object_plan_matches_oracle(k, m, n, lo, hi):
    rng = np.random.default_rng(n + 31 * k + m)
    sizes = [int(x) | 1 for x in rng.integers(max(1, lo // k), hi // k + 1, n)]
    data_np = rng.integers(0, 256, sum(k * s for s in sizes) + 7, dtype=np.uint8)
    data = torch.from_numpy(data_np).cuda()
    parity = torch.full((sum(m * s for s in sizes) + 9,), 0xA5, dtype=torch.uint8, device="cuda")
    objs, offs, do, po = [], [], 3, 5
    for s in sizes:
        objs.append((data.data_ptr() + do, parity.data_ptr() + po, s))
        offs.append((do, po, s))
        do += k * s
        po += m * s
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, objects=objs)
    plan.encode()
    torch.cuda.synchronize()
    pn = parity.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    for i, (do, po, s) in enumerate(offs):
        want = CO.apply(rows, [data_np[do + j * s:do + (j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(pn[po + r * s:po + (r + 1) * s], want[r]), (i, s, r)
    assert (pn[:5] == 0xA5).all() and (pn[po + m * offs[-1][2]:] == 0xA5).all()
    # Reconstruct of a random erasure set on the same plan restores the data
    lost = sorted(rng.choice(k + m, size=m, replace=False).tolist())
    keep = data.clone()
    for do, po, s in offs:
        for i in lost:
            if i < k:
                data[do + i * s:do + (i + 1) * s] = 0x3C
    plan.reconstruct([0 if i in lost else 1 for i in range(k + m)], data_only=True)
    torch.cuda.synchronize()
    assert torch.equal(data, keep)
