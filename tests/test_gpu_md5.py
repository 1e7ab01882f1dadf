"""GPU ShardHash (md5.hip / shardhash.cpp) vs the oracle's shard_hash
(hashlib MD5, objectserver/indexdb.go:746-753) — digest-exact.

Covers the RFC 1321 suite and the reference auditor fixture, every padding
boundary (0, 55, 56, 63, 64, 65, 119, 120 ...), aligned and unaligned views,
>32 views (split launches), partial waves, streaming chains with arbitrary
update sizes (tail carry across updates), multi-stripe shard files, chains of
mixed lengths (md5_list, the host auditor pass), encode+hash with the segment
pipeline, and the batched host path / batcher with hashing.
"""

import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from hummingbird_amd import shardhash as H
from oracle import coracle as CO
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    yield
    torch.cuda.synchronize()


def _dev(b: bytes, pad: int = 0):
    t = torch.zeros(len(b) + pad + 16, dtype=torch.uint8)
    if b:
        t[pad:pad + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
    return t.cuda()


def test_rfc1321_suite(kats):
    for msg, want in kats["md5_rfc1321"]:
        for pad in (0, 1, 3):  # aligned and unaligned starts
            t = _dev(msg.encode(), pad)
            d = H.md5_views([(t.data_ptr() + pad, 0)], 1, len(msg))
            assert H.hexdigests(d)[0] == [want], (msg, pad)


def test_reference_auditor_fixture(kats):
    sh = kats["shard_hash"]
    t = _dev(sh["match"].encode())
    assert H.hexdigests(H.md5_views([(t.data_ptr(), 0)], 1, len(sh["match"])))[0][0] == sh["hash"]
    t = _dev(sh["mismatch"].encode())
    assert H.hexdigests(H.md5_views([(t.data_ptr(), 0)], 1, len(sh["mismatch"])))[0][0] != sh["hash"]


@pytest.mark.parametrize("length", [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1000, 4096, 65536 + 17])
@pytest.mark.parametrize("offset", [0, 5])
def test_batch_lengths(length, offset):
    n_obj, n_views = 130, 3  # 3 waves per view, the last partial
    rng = np.random.default_rng(length * 11 + offset)
    row = n_views * length + offset + 7  # odd row stride when offset/length odd
    host = rng.integers(0, 256, (n_obj, row), dtype=np.uint8)
    t = torch.from_numpy(host).cuda()
    views = [(t.data_ptr() + offset + v * length, row) for v in range(n_views)]
    d = H.hexdigests(H.md5_views(views, n_obj, length))
    for o in range(0, n_obj, 13):
        for v in range(n_views):
            want = O.shard_hash(host[o, offset + v * length: offset + (v + 1) * length])
            assert d[o][v] == want, (o, v)
    # last object (partial wave) fully
    o = n_obj - 1
    assert d[o] == [O.shard_hash(host[o, offset + v * length: offset + (v + 1) * length]) for v in range(n_views)]


def test_many_views_split_launches():
    n_obj, n_views, length = 70, 40, 300
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, (n_obj, n_views * length), dtype=np.uint8)
    t = torch.from_numpy(host).cuda()
    d = H.hexdigests(H.md5_rows(t, n_views, length))
    for o in (0, 33, 69):
        assert d[o] == [O.shard_hash(host[o, v * length:(v + 1) * length]) for v in range(n_views)]


@pytest.mark.parametrize("updates", [[5, 64, 100, 3, 0, 1000, 63, 1], [64] * 5, [4096, 4096, 17],
                                     [1], [0], [], [200_000, 31]])
@pytest.mark.parametrize("offset", [0, 3])
def test_streaming_chains(updates, offset):
    n_obj, n_views = 65, 2
    total = sum(updates)
    rng = np.random.default_rng(len(updates) + total + offset)
    host = rng.integers(0, 256, (n_obj, n_views, total + offset), dtype=np.uint8)
    t = torch.from_numpy(host).cuda()
    row = n_views * (total + offset)
    ch = H.MD5Chains(n_views, n_obj)
    pos = 0
    for u in updates:
        views = [(t.data_ptr() + v * (total + offset) + offset + pos, row) for v in range(n_views)]
        ch.update(views, u)
        pos += u
    d = H.hexdigests(ch.final())
    for o in (0, 31, 64):
        for v in range(n_views):
            assert d[o][v] == O.shard_hash(host[o, v, offset:offset + total]), (o, v)
    # the context resets after final: hash again, one update
    ch.update([(t.data_ptr() + v * (total + offset) + offset, row) for v in range(n_views)], total)
    d2 = H.hexdigests(ch.final())
    assert d2 == d
    ch.close()


@pytest.mark.parametrize("k,m,shard_len,n_obj", [(4, 2, 1 << 18, 24), (4, 2, 1000, 70), (8, 3, 100_000, 9),
                                                (8, 3, 512, 130), (3, 2, 65536, 5), (10, 4, 40_000, 3)])
def test_encode_md5_batch(k, m, shard_len, n_obj):
    enc = RS.New(k, m)
    objs = torch.empty((n_obj, k * shard_len), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * shard_len, first=k * 100 + m)
    parity = torch.empty((n_obj, m * shard_len), dtype=torch.uint8, device="cuda")
    dig = H.encode_objects_md5(enc, objs, parity, shard_len)
    torch.cuda.synchronize()
    host = objs.cpu().numpy()
    par = parity.cpu().numpy()
    want_par = CO.encode_batch(k, m, host)[0] if k <= 16 else None
    got = H.hexdigests(dig)
    for o in sorted({0, n_obj // 2, n_obj - 1}):
        data = [host[o, j * shard_len:(j + 1) * shard_len] for j in range(k)]
        par_o = [par[o, r * shard_len:(r + 1) * shard_len] for r in range(m)]
        if want_par is not None:
            assert np.array_equal(par[o], want_par[o])
        assert got[o] == [O.shard_hash(x) for x in data + par_o], o


def test_multistripe_shard_hash_golden(vectors):
    """A multi-stripe shard file's ShardHash through streaming chains fed one
    stripe's sub-chunks per update (ecutils.go:55-69 concatenation)."""
    v = vectors["shard_hashes_4_2_chunk1k"]
    k, m, chunk = 4, 2, v["chunk"]
    body = bytes(O.object_bytes(v["object"], v["len"]))
    files = O.ec_split(k, m, body, chunk)
    dev = [torch.frombuffer(bytearray(f), dtype=torch.uint8).cuda() for f in files]
    ch = H.MD5Chains(k + m, 1)
    pos, left = 0, v["len"]
    while left > 0:  # per-stripe sub-chunk size (ecutils.go:86-92)
        s = chunk if left >= k * chunk else -(-left // k)
        ch.update([(d.data_ptr() + pos, 0) for d in dev], s)
        pos += s
        left -= min(left, k * s)
    assert H.hexdigests(ch.final())[0] == v["hashes"]


@pytest.mark.parametrize("offset", [0, 3])
def test_md5_list_any_lengths(offset):
    rng = np.random.default_rng(17 + offset)
    lens = [0, 1, 55, 56, 64, 65, 1000, 4096, 70_001, 262_144, 3, 120] * 9  # > 64 chains, mixed waves
    host = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    pool = torch.zeros(sum(n + 32 for n in lens), dtype=torch.uint8, device="cuda")
    bufs, pos = [], 0
    for a in host:
        if a.size:
            pool[pos + offset:pos + offset + a.size] = torch.from_numpy(a).cuda()
        bufs.append((pool.data_ptr() + pos + offset, a.size))
        pos += a.size + 32
    got = [bytes(r).hex() for r in H.md5_list(bufs).cpu().numpy()]
    assert got == [O.shard_hash(a) for a in host]


def test_md5_host_auditor_pass(kats):
    """GPU auditor pass over host 'shard files' of mixed lengths, including the
    reference fixture (auditor_test.go:585-612) and one file larger than a
    staging slot (streamed through a chain)."""
    sh = kats["shard_hash"]
    rng = np.random.default_rng(99)
    files = [sh["match"].encode(), sh["mismatch"].encode(), b""]
    files += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 300_000, 200)]
    files.append(rng.integers(0, 256, (64 << 20) + 4097, dtype=np.uint8).tobytes())
    got = H.md5_host(files)
    assert got[0] == sh["hash"] and got[1] != sh["hash"]
    assert got == [O.shard_hash(f) for f in files]


@pytest.mark.parametrize("k,m,sizes", [(4, 2, [1 << 18] * 40 + [1000, 16, 4096 * 3 + 16]), (8, 3, [512, 1 << 17] * 20),
                                       (3, 2, [7, 100, 65536])])
def test_encode_host_md5(k, m, sizes):
    enc = RS.New(k, m)
    rng = np.random.default_rng(len(sizes) + k)
    stripes = []
    for s in sizes:
        st = np.zeros((k + m) * s, np.uint8)
        st[:k * s] = rng.integers(0, 256, k * s, dtype=np.uint8)
        stripes.append(st)
    hashes = enc.EncodeStripesMD5(stripes)
    mat = CO.build_matrix(k, m)
    for st, s, hs in zip(stripes, sizes, hashes):
        shards = [st[i * s:(i + 1) * s] for i in range(k + m)]
        want = CO.apply(mat[k:], shards[:k])
        for r in range(m):
            assert np.array_equal(shards[k + r], want[r])
        assert hs == [O.shard_hash(x) for x in shards]


def test_batcher_encode_md5_concurrent():
    import threading

    k, m, S = 4, 2, 64 * 1024
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=32 << 20, max_wait_us=300)
    errs = []

    def worker(t):
        try:
            rng = np.random.default_rng(t)
            for _ in range(6):
                st = np.zeros((k + m) * S, np.uint8)
                st[:k * S] = rng.integers(0, 256, k * S, dtype=np.uint8)
                hs = bat.EncodeMD5(st)
                assert hs == [O.shard_hash(st[i * S:(i + 1) * S]) for i in range(k + m)]
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    bat.close()
    assert not errs, errs


def _md5_stats():
    import ctypes as C

    from hummingbird_amd import _native as N

    zc, ring = C.c_uint64(), C.c_uint64()
    assert N.lib().hbec_host_md5_stats(C.byref(zc), C.byref(ring)) == 0
    return zc.value, ring.value


def _pinned_stripes(hb, k, m, sizes, rng):
    """Stripes (ecSplit databuf layout) at 256-B aligned offsets of one
    hbec_host_alloc buffer, data random, parity zero."""
    stripes, off = [], 0
    for s in sizes:
        st = hb.array[off:off + (k + m) * s]
        st[:k * s] = rng.integers(0, 256, k * s, dtype=np.uint8)
        st[k * s:] = 0
        stripes.append(st)
        off += ((k + m) * s + 255) // 256 * 256
    return stripes


def _check_stripes(k, m, sizes, stripes, hashes):
    mat = CO.build_matrix(k, m)
    for st, s, hs in zip(stripes, sizes, hashes):
        shards = [st[i * s:(i + 1) * s] for i in range(k + m)]
        want = CO.apply(mat[k:], shards[:k])
        for r in range(m):
            assert np.array_equal(shards[k + r], want[r])
        assert hs == [O.shard_hash(x) for x in shards]


@pytest.mark.parametrize("k,m,sizes", [(4, 2, [1 << 18] * 40 + [16, 4096 * 3 + 16]), (8, 3, [512, 1 << 17] * 20),
                                       (10, 4, [4096, 65536] * 6), (17, 3, [1024] * 10 + [48]),
                                       (3, 5, [2048, 16, 8192] * 4), (1, 1, [16, 4096])])
def test_encode_host_md5_pinned_zero_copy(k, m, sizes):
    """Pinned stripes: coded in place over PCIe by the mirrored stripes kernel,
    hashed from the device arena (k > 8: accumulate passes; m > 3: output
    groups); parity and every digest against the oracle."""
    enc = RS.New(k, m)
    rng = np.random.default_rng(k * 100 + m)
    total = sum(((k + m) * s + 255) // 256 * 256 for s in sizes)
    hb = RS.HostBuffer(total)
    try:
        stripes = _pinned_stripes(hb, k, m, sizes, rng)
        zc0, ring0 = _md5_stats()
        hashes = enc.EncodeStripesMD5(stripes)
        zc1, ring1 = _md5_stats()
        assert (zc1 - zc0, ring1 - ring0) == (1, 0)
        _check_stripes(k, m, sizes, stripes, hashes)
        del stripes
    finally:
        hb.free()


def test_encode_host_md5_mixed_pinned_and_pageable_takes_ring():
    k, m = 4, 2
    sizes = [4096, 1 << 16, 4096]
    enc = RS.New(k, m)
    rng = np.random.default_rng(5)
    hb = RS.HostBuffer(sum(((k + m) * s + 255) // 256 * 256 for s in sizes))
    try:
        stripes = _pinned_stripes(hb, k, m, sizes, rng)
        page = np.zeros((k + m) * 2048, np.uint8)
        page[:k * 2048] = rng.integers(0, 256, k * 2048, dtype=np.uint8)
        stripes.insert(1, page)
        sizes.insert(1, 2048)
        zc0, ring0 = _md5_stats()
        hashes = enc.EncodeStripesMD5(stripes)
        zc1, ring1 = _md5_stats()
        assert (zc1 - zc0, ring1 - ring0) == (0, 1)
        _check_stripes(k, m, sizes, stripes, hashes)
        del stripes
    finally:
        hb.free()


def test_encode_host_md5_pinned_many_small_stripes_switch_arenas():
    """50 000 pinned 4+2 stripes of 1 KiB shards: 300 000 hash records, more
    than one arena holds (256 K), so arenas alternate mid-batch."""
    k, m, s, n = 4, 2, 1024, 50_000
    enc = RS.New(k, m)
    hb = RS.HostBuffer(n * (k + m) * s)
    try:
        rows = hb.array.reshape(n, (k + m) * s)
        rows[:, :k * s] = np.random.default_rng(11).integers(0, 256, (n, k * s), dtype=np.uint8)
        rows[:, k * s:] = 0
        zc0, _ = _md5_stats()
        hashes = enc.EncodeStripesMD5([rows[i] for i in range(n)])
        assert _md5_stats()[0] == zc0 + 1
        want, _ = CO.encode_batch(k, m, np.ascontiguousarray(rows[:, :k * s]), threads=CO.cpu_threads())
        assert np.array_equal(rows[:, k * s:], want)
        for i in range(0, n, 997):
            assert hashes[i] == [O.shard_hash(rows[i, j * s:(j + 1) * s]) for j in range(k + m)]
        assert hashes[-1] == [O.shard_hash(rows[-1, j * s:(j + 1) * s]) for j in range(k + m)]
        del rows
    finally:
        hb.free()


@pytest.mark.parametrize("k,m,sizes", [
    (4, 2, [(1 << 18) - 1] * 24 + [(1 << 18) - 15, 161, 160, 159, 1, 7, 1001]),
    (8, 3, [131071, 131065, 512 + 3, 200] * 6),
    (10, 4, [104858, 4097, 65537] * 4),   # k > 8: outputs copied to the arena after the last pass
    (17, 3, [1023] * 10 + [49]),
    (3, 5, [2049, 17, 8193] * 4),          # m > 4: two output groups
    (1, 1, [17, 4095])])
def test_encode_host_md5_pinned_unaligned_zero_copy(k, m, sizes):
    """Pinned stripes at odd byte offsets with S % 16 != 0 (ecSplit's S =
    ceil(len / k) for 15 object sizes in 16, objectserver/ecutils.go:14-24):
    coded in place over PCIe by the mirrored gf_odd plan kernel and hashed
    from the device arena: the zero-copy path, parity
    and every digest against the oracle."""
    enc = RS.New(k, m)
    rng = np.random.default_rng(k * 1000 + m)
    total = sum((k + m) * s for s in sizes) + 16 * len(sizes) + 64  # stripes + gaps of < 16 B
    hb = RS.HostBuffer(total)
    try:
        stripes, off = [], 3
        for s in sizes:
            st = hb.array[off:off + (k + m) * s]
            st[:k * s] = rng.integers(0, 256, k * s, dtype=np.uint8)
            st[k * s:] = 0x5A
            stripes.append(st)
            off += (k + m) * s + int(rng.integers(0, 16))
        assert off <= total and all(len(st) == (k + m) * s for st, s in zip(stripes, sizes))
        zc0, ring0 = _md5_stats()
        hashes = enc.EncodeStripesMD5(stripes)
        zc1, ring1 = _md5_stats()
        assert (zc1 - zc0, ring1 - ring0) == (1, 0)
        _check_stripes(k, m, sizes, stripes, hashes)
        del stripes
    finally:
        hb.free()


def test_encode_host_md5_pinned_many_tiny_unaligned_stripes():
    """More pinned, unaligned stripes of S <= 160 than one ring slot holds
    records for (tile_cap = 66 560 at the default 64 MiB slot), k + m = 3.
    Such stripes add an edge record and no main record, so the slot-full test
    must count the edge records too (advisor r03, hostpath.cpp
    zero_copy_unaligned_md5_run): parity and every digest against the oracle."""
    k, m, n = 2, 1, 70_000
    sizes = [(1, 7, 100, 159, 160, 17)[i % 6] for i in range(n)]
    enc = RS.New(k, m)
    rng = np.random.default_rng(99)
    gaps = rng.integers(0, 16, n)
    total = sum((k + m) * s for s in sizes) + int(gaps.sum()) + 64
    hb = RS.HostBuffer(total)
    try:
        stripes, offs, off = [], [], 3
        data = rng.integers(0, 256, total, dtype=np.uint8)
        hb.array[:] = data
        for s, g in zip(sizes, gaps):
            st = hb.array[off:off + (k + m) * s]
            st[k * s:] = 0xA5
            stripes.append(st)
            offs.append(off)
            off += (k + m) * s + int(g)
        zc0, ring0 = _md5_stats()
        hashes = enc.EncodeStripesMD5(stripes)
        zc1, ring1 = _md5_stats()
        assert (zc1 - zc0, ring1 - ring0) == (1, 0)
        for s in sorted(set(sizes)):
            idx = [i for i in range(n) if sizes[i] == s]
            objs = np.stack([np.asarray(stripes[i][:k * s]) for i in idx])
            want, _ = CO.encode_batch(k, m, np.ascontiguousarray(objs))
            got = np.stack([np.asarray(stripes[i][k * s:]) for i in idx])
            assert np.array_equal(got, want), s
        for i in range(n):
            s = sizes[i]
            assert hashes[i] == [O.shard_hash(stripes[i][j * s:(j + 1) * s]) for j in range(k + m)], i
        # bytes between the stripes are untouched
        mask = np.ones(total, bool)
        for o, s in zip(offs, sizes):
            mask[o:o + (k + m) * s] = False
        assert np.array_equal(hb.array[mask], data[mask])
        del stripes
    finally:
        hb.free()
