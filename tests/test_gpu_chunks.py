"""Odd-shard strided batches that cross launch boundaries: a
batch longer than one launch's tiles splits into launches of whole objects
(hbec.cpp odd_launches), each rebuilding its objects' records into the same
scratch and offsetting every base by its first object.  The test hook
hbec_set_odd_chunk_tiles makes a few dozen objects span several launches, so
the table and bit-plane record kernels, gf_odd and the fused guard band run
on objects after the first launch; every parity byte, every rebuilt shard
and every Verify flag is compared with the oracle (reedsolomon.New / Encode /
Reconstruct / Verify, objectserver/ecutils.go:27,59,111)."""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _chunks():
    yield
    B.set_odd_chunk_tiles(0)


# (k, m, S): 8+3 table records, 10+4 / 6+3 bit-plane records, 4+2 gf_odd
@pytest.mark.parametrize("k,m,s", [(8, 3, 8191), (10, 4, 8193), (6, 3, 4099), (4, 2, 6145), (8, 3, 1999)])
def test_odd_batch_across_launches(k, m, s):
    n = 23
    pitch = (k + m) * s + 5
    buf = torch.empty(7 + n * pitch + 64, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(buf.view(1, -1), buf.numel(), first=k * 1000 + s)
    views = [(buf.data_ptr() + 7 + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    B.set_odd_chunk_tiles(40)  # a few objects per launch: 2 to 12 launches per pass
    paths0 = B.odd_path_stats()
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    paths1 = B.odd_path_stats()
    launches = sum(paths1[x] - paths0[x] for x in ("bitplane", "records", "strided"))
    assert launches >= 2, launches
    got = buf.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = 7 + o * pitch
        want = CO.apply(rows, [got[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[b + (k + r) * s:b + (k + r + 1) * s], want[r]), (o, r)
    # the padding between objects is untouched (nothing stored past a shard)
    pads = np.concatenate([got[7 + o * pitch + (k + m) * s:7 + (o + 1) * pitch] for o in range(n)])
    ref = torch.empty_like(buf)
    B.fill_splitmix(ref.view(1, -1), ref.numel(), first=k * 1000 + s)
    refh = ref.cpu().numpy()
    assert np.array_equal(pads, np.concatenate([refh[7 + o * pitch + (k + m) * s:7 + (o + 1) * pitch]
                                                for o in range(n)]))
    # three shards lost (data and parity), rebuilt across the same launches
    keep = buf.clone()
    lost = [0, k - 1, k + m - 1][:m]
    for o in range(n):
        for i in lost:
            a = 7 + o * pitch + i * s
            buf[a:a + s] = 0x5A
    B.reconstruct_views(enc, views, [0 if i in lost else 1 for i in range(k + m)], n, s)
    torch.cuda.synchronize()
    assert torch.equal(buf, keep)
    # Verify: clean, then flips in objects of later launches flag exactly them
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0
    hit = {6: (k, 0), 13: (0, s - 1), 22: (k + m - 1, s // 2)}
    for o, (i, p) in hit.items():
        buf[7 + o * pitch + i * s + p] ^= 0x40
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == sorted(hit)
