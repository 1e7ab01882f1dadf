"""GPU parity of the 16-B-aligned views that apply_views routes to the record
kernels (csrc/hbec.cpp rec_route): 9 <= k <= 12 at any pitch and
5 <= k <= 8 when a base, object stride or S is not a multiple of the 128-B
line; k <= 4 and line-aligned 5 <= k <= 8 stay on the aligned kernels.

ecSplit databufs (shard i at i*S, objectserver/ecutils.go:31-35) at 16-B
but not 128-B aligned pitches and at 128-B pitches: Encode (ecutils.go:59)
and Reconstruct of two data shards (ecutils.go:111) against the oracle, byte
for byte, and the route taken read from hbec_odd_path_stats.
"""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

import route_rule as R

pytestmark = pytest.mark.gpu


def _odd_launches():
    p = B.odd_path_stats()
    return p["bitplane"] + p["records"] + p["strided"]


def _routed(k, m, s, base):
    from hummingbird_amd import gen_xor
    return R.rec_route(k, s, base, rows=m, bitplane=gen_xor.USE.get((k, m), (False,))[0])


def test_route_rule_thresholds():
    """the mirror reads tuning.h: 24 KiB for 9 <= k <= 12, 48 KiB off the line for 5 <= k <= 8"""
    assert (R.MIN_S_BIG, R.MIN_S) == (24576, 49152)


@pytest.mark.parametrize("k,m,s,off", [(8, 3, 49168, 0), (8, 3, 49152, 16), (8, 3, 49152, 0), (6, 4, 49200, 0),
                                       (5, 3, 61456, 48), (7, 3, 8208, 0), (9, 3, 24592, 0), (10, 4, 24576, 0),
                                       (12, 4, 32768, 0), (12, 3, 26640, 32), (10, 2, 24560, 0), (4, 2, 65552, 0),
                                       (4, 2, 65536, 0), (8, 4, 65552, 0), (8, 3, 4112, 0), (8, 4, 65536, 0),
                                       (6, 4, 49152, 0), (7, 4, 65536, 0), (7, 4, 65552, 0), (6, 6, 49152, 0)])
def test_aligned_views_route_and_parity(k, m, s, off):
    n = max(3, min(48, 3_000_000 // ((k + m) * s)))
    pitch = (k + m) * s
    buf = torch.empty(off + n * pitch + 64, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(buf.view(1, -1), buf.numel())
    base = buf.data_ptr() + off
    views = [(base + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    before = _odd_launches()
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    assert (_odd_launches() > before) == _routed(k, m, s, base), "route"
    got = buf.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = off + o * pitch
        want = CO.apply(rows, [got[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[b + (k + r) * s:b + (k + r + 1) * s], want[r]), (o, r)
    # two data shards lost: rebuilt in place from the first k survivors
    ref = buf.clone()
    for o in range(n):
        buf[off + o * pitch:off + o * pitch + 2 * s] = 0xA5
    before = _odd_launches()
    B.reconstruct_views(enc, views, [0, 0] + [1] * (k + m - 2), n, s)
    torch.cuda.synchronize()
    assert (_odd_launches() > before) == R.rec_route(k, s, base, rows=2), "route (reconstruct)"
    assert torch.equal(buf, ref)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    before = _odd_launches()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0
    # Verify: gf_verify_pipe (k <= 8, m <= 4) except past K R = 24 with a
    # compiled bit-plane Verify (8+4); everything else on the odd kernels
    from hummingbird_amd import gen_xor
    v_rec = 5 <= k <= 8 and k * m > 24 and m <= 4 and s >= R.MIN_S and gen_xor.USE.get((k, m), (0, 0, 0))[2]
    assert (_odd_launches() > before) == (bool(v_rec) or 9 <= k <= 12 or m > 4), "route (Verify)"
    # a flipped parity byte is caught on either route
    buf[off + (n - 1) * pitch + k * s + s // 2] ^= 1
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == [n - 1]


def test_kernel_info_reports_the_route():
    assert B.kernel_info(4, 2, 1 << 18)["kind"] == "pipelined"
    assert B.kernel_info(8, 3, 1 << 17)["kind"] == "pipelined"
    assert B.kernel_info(8, 3, (1 << 17) + 16)["kind"] == "records"
    assert B.kernel_info(8, 3, 4096 + 16)["kind"] == "packed"  # 5 <= k <= 8 packed to 32 KiB (round 6)
    assert B.kernel_info(8, 3, 32768 + 16)["kind"] == "pipelined"
    assert B.kernel_info(10, 4, 1 << 17)["kind"] == "records"
    assert B.kernel_info(10, 4, 1 << 14)["kind"] == "streaming"  # the aligned k > 8 kernel
    assert B.kernel_info(8, 3, 512)["kind"] == "packed"


@pytest.mark.parametrize("k,m,s", [(10, 5, 24577), (9, 6, 8193), (12, 5, 32768), (11, 8, 4099)])
def test_verify_wide_route_9_12_more_than_4_rows(k, m, s):
    """Verify of 9 <= k <= 12 with m > 4 parity rows takes
    gf_verify_wide (one read-only pass per <= 8 rows, hbec.cpp verify_views),
    not the odd kernels: oracle parity passes clean, and single-byte flips in
    the first and last parity row and in a data shard flag exactly their
    objects."""
    n = 9
    pitch = (k + m) * s + 16
    buf = torch.empty(n * pitch + 64, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(buf.view(1, -1), buf.numel(), first=k * 100 + m)
    host = buf.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = 3 + o * pitch
        want = CO.apply(rows, [host[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            host[b + (k + r) * s:b + (k + r + 1) * s] = want[r]
    buf.copy_(torch.from_numpy(host))
    views = [(buf.data_ptr() + 3 + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    before = _odd_launches()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert _odd_launches() == before, "m > 4 rows: gf_verify_wide"
    assert int(flags.count_nonzero()) == 0
    hits = {1: (k, 0), 4: (k + m - 1, s - 1), 7: (k // 2, s // 2)}  # object: (shard, byte)
    for o, (i, p) in hits.items():
        buf[3 + o * pitch + i * s + p] ^= 0x11
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == sorted(hits)


# Round 6: gf_odd (k <= 4, <= 3 outputs) codes each shard's guard band (the
# <= 64 head and tail bytes outside its 16-B frame) in the shard's first and
# last tile (tuning.h HBEC_ODD_EDGE_FUSE); shards of one frame tile, the
# record kernels and Verify keep the gf_odd_edges launch.
@pytest.mark.parametrize("k,m,s,fused", [(4, 2, 4095, True), (3, 2, 8191, True), (2, 1, 100003, True),
                                         (1, 3, 6001, True), (4, 3, 2301, True), (4, 2, 2047, False),
                                         (8, 3, 8191, False), (10, 4, 8193, False)])
def test_guard_band_fused_route_and_parity(k, m, s, fused):
    n = 37
    pitch = (k + m) * s + 3
    buf = torch.empty(5 + n * pitch + 64, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(buf.view(1, -1), buf.numel(), first=s)
    ref = buf.clone()
    views = [(buf.data_ptr() + 5 + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    p0 = B.odd_path_stats()
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    p1 = B.odd_path_stats()
    assert (p1["fused"] > p0["fused"], p1["edges"] > p0["edges"]) == (fused, not fused)
    got = buf.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = 5 + o * pitch
        want = CO.apply(rows, [got[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[b + (k + r) * s:b + (k + r + 1) * s], want[r]), (o, r)
    # nothing outside the shards changed (the guard-band stores are byte-exact)
    refh = ref.cpu().numpy()
    gaps = [(0, 5)] + [(5 + o * pitch + (k + m) * s, 5 + (o + 1) * pitch) for o in range(n)]
    gaps.append((5 + n * pitch, refh.size))
    for a, e in gaps:
        assert np.array_equal(got[a:e], refh[a:e])
    # min(2, m) shards lost and rebuilt (gf_odd again for k <= 4)
    keep = buf.clone()
    lost = ([0, k] if k > 1 else [0, 1])[:m]
    for o in range(n):
        for i in lost:
            a = 5 + o * pitch + i * s
            buf[a:a + s] = 0xA5
    B.reconstruct_views(enc, views, [0 if i in lost else 1 for i in range(k + m)], n, s)
    torch.cuda.synchronize()
    assert torch.equal(buf, keep)
