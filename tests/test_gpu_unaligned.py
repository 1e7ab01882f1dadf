"""GPU parity of gf_apply_unaligned (kernels.hip): views at any byte offset,
any object stride, any shard length.

ecSplit sets S = ceil(len / k) (objectserver/ecutils.go:14-24) and puts
shard i of its databuf at i*S (ecutils.go:31-35), so an arbitrary object's
shards start at arbitrary byte offsets; this kernel codes them with aligned
16-B accesses and in-register shifts.  Every case compares with the oracle
(oracle/coracle.py, klauspost's algorithm) byte for byte and checks that no
byte outside the output views changed (head / tail blocks are stored
bytewise; a stray 16-B store would show up in the guard bytes).
"""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

import route_rule as R

pytestmark = pytest.mark.gpu
GUARD = 0xA5

LENGTHS = [1, 3, 15, 16, 17, 63, 64, 1000, 1007, 1008, 1009, 2015, 2016, 2017, 4031, 4033, 4096, 5000, 65537]


def _cases():
    rng = np.random.default_rng(20261017)
    for i in range(48):
        rows = int(rng.choice([1, 2, 3, 4, 5, 6]))
        cols = int(rng.choice([1, 2, 3, 4, 6, 8, 10, 16, 17, 20]))
        s = int(LENGTHS[i % len(LENGTHS)])
        n = int(rng.choice([1, 2, 5, 9]))
        yield rows, cols, s, n, int(rng.integers(0, 1 << 30))


def _run_apply(rows, cols, s, n, seed):
    rng = np.random.default_rng(seed)
    coeffs = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    special = rng.random((rows, cols))
    coeffs[special < 0.15] = 0
    coeffs[(special >= 0.15) & (special < 0.3)] = 1
    in_off, out_off = int(rng.integers(0, 16)), int(rng.integers(0, 16))
    in_stride = cols * s + int(rng.integers(0, 32))
    out_stride = rows * s + int(rng.integers(0, 32))
    in_np = rng.integers(0, 256, in_off + n * in_stride + 16, dtype=np.uint8)
    ins = torch.from_numpy(in_np).cuda()
    outs = torch.full((out_off + n * out_stride + 16,), GUARD, dtype=torch.uint8, device="cuda")
    iv = [(ins.data_ptr() + in_off + c * s, in_stride) for c in range(cols)]
    ov = [(outs.data_ptr() + out_off + r * s, out_stride) for r in range(rows)]
    B.apply_views(rows, cols, coeffs.tolist(), iv, ov, n, s)
    torch.cuda.synchronize()
    got = outs.cpu().numpy()
    want = np.full_like(got, GUARD)
    for o in range(n):
        b = in_off + o * in_stride
        res = CO.apply(coeffs, [in_np[b + c * s:b + (c + 1) * s] for c in range(cols)])
        for r in range(rows):
            a = out_off + o * out_stride + r * s
            want[a:a + s] = res[r]
    return got, want


@pytest.mark.parametrize("rows,cols,s,n,seed", list(_cases()))
def test_unaligned_apply_matches_oracle(rows, cols, s, n, seed):
    """Random odd offsets / strides / lengths (1 B .. 64 KiB, inputs 1..20 so
    the k > 16 accumulate pass is unaligned too, outputs 1..6 so > 4 rows
    take a second pass) against the oracle, guard bytes untouched."""
    got, want = _run_apply(rows, cols, s, n, seed)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


@pytest.mark.parametrize("off_in,off_out", [(0, 1), (1, 0), (5, 5), (15, 3), (8, 12)])
def test_unaligned_every_offset_pair(off_in, off_out):
    """Fixed offset pairs, including equal misalignment of input and output
    and an aligned input with an unaligned output (and the reverse)."""
    k, m, n, s = 4, 2, 3, 3001
    rng = np.random.default_rng(off_in * 16 + off_out)
    enc_rows = CO.build_matrix(k, m)[k:]
    in_np = rng.integers(0, 256, off_in + n * k * s + 16, dtype=np.uint8)
    ins = torch.from_numpy(in_np).cuda()
    outs = torch.full((off_out + n * m * s + 16,), GUARD, dtype=torch.uint8, device="cuda")
    iv = [(ins.data_ptr() + off_in + j * s, k * s) for j in range(k)]
    ov = [(outs.data_ptr() + off_out + r * s, m * s) for r in range(m)]
    B.apply_views(m, k, enc_rows.tolist(), iv, ov, n, s)
    torch.cuda.synchronize()
    got = outs.cpu().numpy()
    want = np.full_like(got, GUARD)
    for o in range(n):
        b = off_in + o * k * s
        res = CO.apply(enc_rows, [in_np[b + j * s:b + (j + 1) * s] for j in range(k)])
        for r in range(m):
            a = off_out + (o * m + r) * s
            want[a:a + s] = res[r]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k,m,obj_len,n", [(4, 2, (1 << 20) - 4, 8), (4, 2, 1000001, 8), (8, 3, (1 << 20) - 8, 8),
                                           (6, 3, 1 << 20, 8), (10, 4, 1 << 20, 8), (3, 2, 7, 8),
                                           # several tiles per wave (the record prefetch runs ahead):
                                           # 12+4 / 11+4 / 9+4 with coefficient tables in LDS, 8+4
                                           # and 8+3 register-resident, 24+4 with a 12-input
                                           # accumulate pass
                                           (12, 4, 12 * 87389, 160), (11, 4, (1 << 20) - 3, 160),
                                           (9, 4, (1 << 20) + 5, 160), (8, 4, (1 << 20) - 8, 160),
                                           (8, 3, (1 << 20) - 8, 200), (4, 2, (1 << 20) - 4, 200),
                                           (6, 3, (1 << 20) + 3, 160), (7, 3, (1 << 20) - 5, 120),
                                           (24, 4, (1 << 20) - 7, 96)])
def test_databuf_odd_shards_encode_reconstruct(k, m, obj_len, n):
    """ecSplit databufs of objects whose size gives S % 16 != 0 (shard i at
    i*S, rows of (k+m)*S): Encode against the oracle, then Reconstruct and
    ReconstructData of random erasures restore every shard."""
    s = -(-obj_len // k)
    rng = np.random.default_rng(obj_len + k)
    rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(rows, (k + m) * s, first=obj_len)
    enc = RS.New(k, m)
    views = B.shard_views(rows, k + m, s)
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    r_np = rows.cpu().numpy()
    par_rows = CO.build_matrix(k, m)[k:]
    for o in range(n):
        want = CO.apply(par_rows, [r_np[o, j * s:(j + 1) * s] for j in range(k)])
        for r in range(m):
            assert np.array_equal(r_np[o, (k + r) * s:(k + r + 1) * s], want[r]), (o, r)
    for data_only in (False, True):
        lost = sorted(rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False).tolist())
        damaged = rows.clone()
        for i in lost:
            damaged[:, i * s:(i + 1) * s] = 0x3C
        B.reconstruct_views(enc, B.shard_views(damaged, k + m, s), [0 if i in lost else 1 for i in range(k + m)],
                            n, s, data_only=data_only)
        torch.cuda.synchronize()
        d = damaged.cpu().numpy()
        for i in range(k + m):
            if data_only and i >= k and i in lost:
                assert (d[:, i * s:(i + 1) * s] == 0x3C).all()
            else:
                assert np.array_equal(d[:, i * s:(i + 1) * s], r_np[:, i * s:(i + 1) * s]), (lost, i, data_only)


def test_unaligned_large_batch_verify():
    """256 objects of 1 MiB - 4 B (S = 262 143) in 4+2 databufs: Encode, then
    Verify (a different kernel) passes on every object, and a flipped byte in
    the last shard's tail is flagged on that object only."""
    k, m, n = 4, 2, 256
    s = ((1 << 20) - 4) // k
    rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(rows, (k + m) * s)
    enc = RS.New(k, m)
    views = B.shard_views(rows, k + m, s)
    B.encode_views(enc, views, n, s)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero().item()) == 0
    rows[77, (k + m) * s - 1] ^= 1
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == [77]


@pytest.mark.parametrize("k,m,n,lo,hi", [(4, 2, 300, 1, 200_000), (8, 3, 120, 1, 200_000), (12, 4, 60, 1, 200_000),
                                         (20, 4, 24, 1, 200_000), (5, 5, 40, 1, 200_000),
                                         (4, 2, 100, 150_000, 150_900), (8, 3, 60, 300_000, 301_000),
                                         (12, 4, 40, 500_000, 500_100), (20, 4, 12, 400_000, 401_000)])
def test_plan_random_odd_stripes(k, m, n, lo, hi):
    """Stripe plans whose stripes have random sizes (S % 16 != 0) at random
    byte offsets, coded in one launch per pass (k = 20: an accumulate pass;
    m = 5: two output passes): sizes over [1, 200 000) take per-window
    records (gf_odd_plan), near-uniform sizes per-stripe records (gf_odd_rec).
    Encode and Reconstruct of a random erasure set match the oracle; bytes
    between stripes are untouched."""
    rng = np.random.default_rng(k * 1000 + m * 10 + n)
    layout, off = [], 0
    for _ in range(n):
        size = int(rng.integers(lo, hi))
        s = -(-size // k)
        off += int(rng.integers(1, 40))
        layout.append((off, s))
        off += (k + m) * s
    pool = rng.integers(0, 256, off + 64, dtype=np.uint8)
    mat = CO.build_matrix(k, m)[k:]
    want = pool.copy()
    for o, s in layout:
        for r, p in enumerate(CO.apply(mat, [want[o + j * s:o + (j + 1) * s] for j in range(k)])):
            want[o + (k + r) * s:o + (k + r + 1) * s] = p
    dev = torch.from_numpy(pool).cuda()
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, [(dev.data_ptr() + o, s) for o, s in layout])
    assert plan.info()["n_fallback"] == sum(R.stripe_on_records(k, m, dev.data_ptr() + o, s) for o, s in layout)
    plan.encode()
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    lost = sorted(rng.choice(k + m, size=m, replace=False).tolist())
    damaged = torch.from_numpy(want.copy()).cuda()
    for o, s in layout:
        for i in lost:
            damaged[o + i * s:o + (i + 1) * s] = 0xEE
    B.StripePlan(enc, [(damaged.data_ptr() + o, s) for o, s in layout]).reconstruct(
        [0 if i in lost else 1 for i in range(k + m)])
    torch.cuda.synchronize()
    assert np.array_equal(damaged.cpu().numpy(), want), lost


@pytest.mark.parametrize("k,m,clusters", [(4, 2, ((3000, 3100), (300_000, 300_900))),
                                          (8, 3, ((5000, 5100), (1 << 20, (1 << 20) + 500), (1, 900))),
                                          (12, 4, ((60_000, 60_400), (600_000, 601_000))),
                                          (20, 4, ((40_000, 40_500), (400_000, 400_800)))])
def test_plan_clustered_odd_stripes(k, m, clusters):
    """Stripe plans whose odd-sized stripes fall into a few size classes
    (small and large objects, plus a class of tiny stripes that only the edge
    kernel codes): one per-stripe-record launch per class, stripes of the
    classes interleaved in the plan.  Encode and Reconstruct against the
    oracle; bytes between stripes untouched."""
    rng = np.random.default_rng(k * 7 + m)
    layout, off = [], 0
    for i in range(48):
        lo, hi = clusters[i % len(clusters)]
        s = -(-int(rng.integers(lo, hi)) // k)
        off += int(rng.integers(1, 40))
        layout.append((off, s))
        off += (k + m) * s
    pool = rng.integers(0, 256, off + 64, dtype=np.uint8)
    mat = CO.build_matrix(k, m)[k:]
    want = pool.copy()
    for o, s in layout:
        for r, p in enumerate(CO.apply(mat, [want[o + j * s:o + (j + 1) * s] for j in range(k)])):
            want[o + (k + r) * s:o + (k + r + 1) * s] = p
    dev = torch.from_numpy(pool).cuda()
    enc = RS.New(k, m)
    B.StripePlan(enc, [(dev.data_ptr() + o, s) for o, s in layout]).encode()
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    lost = sorted(rng.choice(k + m, size=m, replace=False).tolist())
    damaged = torch.from_numpy(want.copy()).cuda()
    for o, s in layout:
        for i in lost:
            damaged[o + i * s:o + (i + 1) * s] = 0xEE
    B.StripePlan(enc, [(damaged.data_ptr() + o, s) for o, s in layout]).reconstruct(
        [0 if i in lost else 1 for i in range(k + m)])
    torch.cuda.synchronize()
    assert np.array_equal(damaged.cpu().numpy(), want), lost


@pytest.mark.parametrize("k,m", [(4, 2), (8, 3), (10, 4), (20, 4)])
def test_host_pinned_odd_stripes_zero_copy(k, m):
    """Pinned host stripes of odd sizes at odd byte offsets (ecSplit databufs
    of arbitrary objects in a hbec_host_alloc pool): coded in place over PCIe
    by the unaligned kernel, through the batched host path and through the
    per-call databuf entry, against the oracle; bytes between stripes are
    untouched."""
    from oracle import oracle as O

    rng = np.random.default_rng(k * 7 + m)
    sizes = [int(x) for x in rng.integers(1, 300_000, size=24)] + [(1 << 20) - 3, 1001, 7]
    layout, off = [], 0
    for size in sizes:
        s = O.ec_shard_length(size, k)
        off += int(rng.integers(1, 16))
        layout.append((off, s, size))
        off += (k + m) * s
    hb = RS.HostBuffer(off + 64)
    a = hb.array
    a[:] = GUARD
    for i, (o, s, size) in enumerate(layout):
        a[o:o + (k + m) * s] = 0
        a[o:o + size] = CO.fill_objects(300 + i, 1, size)[0]
    want = a.copy()
    mat = CO.build_matrix(k, m)[k:]
    for o, s, _ in layout:
        for r, p in enumerate(CO.apply(mat, [want[o + j * s:o + (j + 1) * s] for j in range(k)])):
            want[o + (k + r) * s:o + (k + r + 1) * s] = p
    enc = RS.New(k, m)
    stripes = [a[o:o + (k + m) * s] for o, s, _ in layout]
    assert all(RS.host_device_addr(st) != 0 for st in stripes)
    enc.EncodeStripes(stripes)
    assert np.array_equal(a, want)
    lost = sorted(rng.choice(k + m, size=m, replace=False).tolist())
    for o, s, _ in layout:
        for i in lost:
            a[o + i * s:o + (i + 1) * s] = 0x5A
    enc.ReconstructStripes(stripes, [0 if i in lost else 1 for i in range(k + m)])
    assert np.array_equal(a, want), lost
    # per-call databuf entries (the cgo shim's path), one stripe per call
    for o, s, _ in layout:
        a[o + k * s:o + (k + m) * s] = 0x77
    for st, (o, s, _) in zip(stripes, layout):
        enc.EncodeDatabuf(st, s)
    assert np.array_equal(a, want)
    for st, (o, s, _) in zip(stripes, layout):
        st[:s] = 0x11
        enc.ReconstructDatabuf(st, s, [0] + [1] * (k + m - 1))
    assert np.array_equal(a, want)
    del stripes
    hb.free()


@pytest.mark.parametrize("k,m,s,off,n", [(4, 2, 1001, 3, 12), (8, 3, 131071, 0, 12), (6, 3, 17, 5, 12),
                                         (10, 4, 104858, 1, 12), (16, 6, 2015, 9, 12), (17, 3, 333, 2, 12),
                                         (3, 2, 1, 15, 12),
                                         # gf_verify_wide (k > 12)
                                         (20, 4, 52429, 3, 12), (32, 8, 32768, 0, 12), (32, 8, 4097, 7, 12),
                                         (20, 4, 31, 1, 12), (12, 9, 1000, 2, 12), (9, 1, 48, 0, 12),
                                         (64, 4, 16387, 5, 12),
                                         # chained 4-window Verify tiles (K <= 4), several tiles per wave
                                         (4, 2, 262143, 5, 160), (2, 2, 100003, 1, 96), (3, 1, 4081, 11, 200),
                                         # record kernel with LDS tables, several tiles per wave
                                         (10, 4, 104858, 7, 160), (12, 4, 87389, 2, 160), (11, 3, 95325, 9, 96),
                                         (9, 2, 116509, 0, 96),
                                         # 9 <= k <= 12 with R <= 2: gf_odd's register-table Verify
                                         (9, 1, 30001, 3, 64), (11, 2, 50001, 4, 64), (12, 1, 7777, 1, 64)])
def test_unaligned_verify_flags_exactly(k, m, s, off, n):
    """Encoder.Verify over unaligned views (gf_odd verify for k <= 8, the
    record kernel for 9 <= k <= 12, gf_verify_wide above: one read-only pass
    for any k): clean codewords from the oracle are not flagged; a flipped
    first / last / middle byte of a parity shard, or of a data shard, flags
    exactly that object."""
    rng = np.random.default_rng(k * 1000 + s)
    row = (k + m) * s + 5
    buf = rng.integers(0, 256, off + n * row + 16, dtype=np.uint8)
    mat = CO.build_matrix(k, m)[k:]
    for o in range(n):
        b = off + o * row
        for r, p in enumerate(CO.apply(mat, [buf[b + j * s:b + (j + 1) * s] for j in range(k)])):
            buf[b + (k + r) * s:b + (k + r + 1) * s] = p
    dev = torch.from_numpy(buf).cuda()
    views = [(dev.data_ptr() + off + i * s, row) for i in range(k + m)]
    enc = RS.New(k, m)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero().item()) == 0
    flips = {1: off + 1 * row + k * s,                      # first byte of parity 0
             4: off + 4 * row + (k + m) * s - 1,            # last byte of the last parity shard
             7: off + 7 * row + (k + m - 1) * s + s // 2,   # middle of the last parity shard
             10: off + 10 * row + s - 1}                    # last byte of data shard 0
    for pos in flips.values():
        dev[pos] ^= 0x40
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == sorted(flips)
