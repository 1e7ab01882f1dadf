"""GPU parity of the bit-plane record kernels (odd_impl.h bp_dot2, the
compiled XOR networks of xor_sched.h): odd-shard encodes of every compiled
(k, m) against the oracle, byte for byte.

The encode matrix is reedsolomon.New(k, m)'s parity rows
(objectserver/ecutils.go:27,59); a pass whose coefficients equal a compiled
schedule takes the bit-plane kernel (hbec_odd_path_stats counts it), every
other pass the v_perm table kernels.  Shards at odd offsets and of odd
lengths (ecSplit's S = ceil(len / k), ecutils.go:14-24, databuf slots at i*S,
ecutils.go:31-35), several tiles per wave, guard bytes around every output.
"""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import gen_xor
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu
GUARD = 0x5A

SHAPES = gen_xor.SHAPES


def _bp():
    return B.odd_path_stats()["bitplane"]


@pytest.mark.parametrize("k,m", SHAPES)
@pytest.mark.parametrize("s", [161, 1001, 2017, 4033, 20011])
def test_bitplane_encode_split_layout(k, m, s):
    """Separate data / parity arrays at odd offsets and pitches: every parity
    byte equals the oracle's, the guard bytes around each output survive."""
    n = max(3, min(64, 4_000_000 // ((k + m) * s)))
    rng = np.random.default_rng(k * 1000 + m * 100 + s)
    in_off, out_off = int(rng.integers(1, 16)), int(rng.integers(0, 16))
    in_stride, out_stride = k * s + int(rng.integers(0, 40)), m * s + int(rng.integers(1, 40))
    in_np = rng.integers(0, 256, in_off + n * in_stride + 16, dtype=np.uint8)
    ins = torch.from_numpy(in_np).cuda()
    outs = torch.full((out_off + n * out_stride + 16,), GUARD, dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    iv = [(ins.data_ptr() + in_off + j * s, in_stride) for j in range(k)]
    ov = [(outs.data_ptr() + out_off + r * s, out_stride) for r in range(m)]
    before = _bp()
    B.encode_views(enc, iv + ov, n, s)
    torch.cuda.synchronize()
    # strided batches take the bit-plane kernel where it measured faster
    assert (_bp() > before) == gen_xor.USE[(k, m)][0]
    got = outs.cpu().numpy()
    want = np.full_like(got, GUARD)
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = in_off + o * in_stride
        res = CO.apply(rows, [in_np[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            a = out_off + o * out_stride + r * s
            want[a:a + s] = res[r]
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


@pytest.mark.parametrize("k,m,obj_len,n", [(9, 3, (1 << 20) - 8, 160), (10, 4, 1 << 20, 160),
                                           (12, 4, 12 * 87389, 128), (6, 3, (1 << 20) + 3, 160),
                                           (8, 2, (1 << 20) - 9, 64), (8, 4, (1 << 20) - 9, 96)])
def test_bitplane_databuf_many_tiles_then_rebuild(k, m, obj_len, n):
    """ecSplit databufs of 1 MiB-class objects (many tiles per wave, so the
    record prefetch runs ahead): Encode against the oracle, then a
    parity-only Reconstruct (the same parity rows: bit-plane again) restores
    the parity shards exactly."""
    s = -(-obj_len // k)
    rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(rows, (k + m) * s, first=obj_len)
    enc = RS.New(k, m)
    views = B.shard_views(rows, k + m, s)
    before = _bp()
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    assert (_bp() > before) == gen_xor.USE[(k, m)][0]
    r_np = rows.cpu().numpy()
    par = CO.build_matrix(k, m)[k:]
    for o in range(n):
        want = CO.apply(par, [r_np[o, j * s:(j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(r_np[o, (k + r) * s:(k + r + 1) * s], want[r]), (o, r)
    damaged = rows.clone()
    damaged[:, k * s:] = 0x3C
    before = _bp()
    B.reconstruct_views(enc, B.shard_views(damaged, k + m, s), [1] * k + [0] * m, n, s)
    torch.cuda.synchronize()
    assert (_bp() > before) == gen_xor.USE[(k, m)][0]
    assert torch.equal(damaged, rows)


@pytest.mark.parametrize("k,m", [km for km in SHAPES if gen_xor.USE[km][1]])
def test_bitplane_object_plan(k, m):
    """Object plans of near-uniform odd sizes (per-stripe records, one class)
    take the bit-plane kernel too; every parity byte against the oracle."""
    rng = np.random.default_rng(k + m)
    n = 64
    sizes = [int(x) for x in rng.integers(60_001, 60_400, n)]
    d = torch.empty(sum(k * x for x in sizes) + 16, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(d.view(1, -1), d.numel())
    par = torch.full((sum(m * x for x in sizes) + 16,), GUARD, dtype=torch.uint8, device="cuda")
    objs, do, po = [], 3, 5
    for x in sizes:
        objs.append((d.data_ptr() + do, par.data_ptr() + po, x))
        do += k * x
        po += m * x
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, objects=objs)
    before = _bp()
    plan.encode()
    torch.cuda.synchronize()
    assert _bp() > before
    dn, pn = d.cpu().numpy(), par.cpu().numpy()
    rows = CO.build_matrix(k, m)[k:]
    do, po = 3, 5
    for x in sizes:
        want = CO.apply(rows, [dn[do + j * x:do + (j + 1) * x] for j in range(k)])
        for r in range(m):
            assert np.array_equal(pn[po + r * x:po + (r + 1) * x], want[r])
        do += k * x
        po += m * x
    assert (pn[:5] == GUARD).all() and (pn[po:] == GUARD).all()


@pytest.mark.parametrize("k,m,s", [(km[0], km[1], s) for km in SHAPES if gen_xor.USE[km][2]
                                   for s in (161, 2031, 2033, 20011)])
def test_bitplane_verify_flags_exactly(k, m, s):
    """Verify through the chained bit-plane kernel (2 windows per tile, the
    last column of window 0 borrowing window 1's first dword): oracle
    codewords at odd offsets pass, and a single flipped byte — anywhere,
    including next to the 2032-B tile boundaries and the window seam — flags
    exactly its object."""
    n = 24
    rng = np.random.default_rng(7 * k + m + s)
    off = int(rng.integers(1, 16))
    pitch = (k + m) * s + 5
    buf_np = rng.integers(0, 256, off + n * pitch + 16, dtype=np.uint8)
    rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = off + o * pitch
        par = CO.apply(rows, [buf_np[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            buf_np[b + (k + r) * s:b + (k + r + 1) * s] = par[r]
    buf = torch.from_numpy(buf_np).cuda()
    views = [(buf.data_ptr() + off + i * s, pitch) for i in range(k + m)]
    enc = RS.New(k, m)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    before = _bp()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert _bp() > before, "the bit-plane Verify did not run"
    assert int(flags.count_nonzero()) == 0
    # flips: object -> (shard, position)
    cand = sorted({p for t in range(1, s // 2032 + 2) for p in (2032 * t - 2, 2032 * t - 1, 2032 * t, 2032 * t + 15)
                   if 0 <= p < s} | {0, s - 1, min(s - 1, 1023), min(s - 1, 1024), min(s - 1, 1008)})
    hit = {}
    for o in range(0, n, 2):
        hit[o] = (int(rng.integers(0, k + m)), cand[(o // 2) % len(cand)])
    for o, (i, p) in hit.items():
        buf[off + o * pitch + i * s + p] ^= 0x10
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert sorted(flags.nonzero().flatten().tolist()) == sorted(hit)
