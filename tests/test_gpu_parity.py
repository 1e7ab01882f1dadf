"""GPU parity: libhbec's HIP kernels vs the CPU oracle (bit-exact).

Everything here calls through the C ABI (include/hbec.h) and runs the gfx950
kernels.  Checks mirror what the reference path computes:
  * klauspost Encoder semantics (Encode / Reconstruct / ReconstructData) on
    the upstream KAT and on random shards of many shapes (vec path, byte path,
    >16 inputs, >4 outputs),
  * every erasure pattern of 4+2 and 8+3 (golden digests),
  * the ecutils stripe loops (ecSplit / ecReconstruct / ecGlue) against the
    golden shard files, including padding and multi-stripe objects,
  * device batches at 64 x 1 MiB and at the BASELINE size 4096 x 1 MiB
    (every object compared with the oracle).
"""
import hashlib
import io
import itertools

import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import ecutils as E
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO
from oracle import oracle as O

import route_rule as R

pytestmark = pytest.mark.gpu
MiB = 1 << 20


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.init()
    yield
    torch.cuda.synchronize()


def test_one_encode_kat(kats):
    c = kats["one_encode"]
    enc = RS.New(c["k"], c["m"])
    shards = [np.array(d, np.uint8) for d in c["data"]] + [np.zeros(2, np.uint8) for _ in range(c["m"])]
    enc.Encode(shards)
    assert [s.tolist() for s in shards[c["k"]:]] == c["parity"]


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (3, 2), (4, 2), (5, 5), (8, 3), (10, 4), (16, 4), (17, 3),
                                 (12, 6), (20, 8), (100, 20)])
@pytest.mark.parametrize("n", [1, 3, 16, 17, 1000, 4096, 65536 + 5])
def test_encode_matches_oracle(k, m, n):
    rng = np.random.default_rng(k * 7919 + m * 31 + n)
    enc = RS.New(k, m)
    shards = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8)
                                                                          for _ in range(m)]
    enc.Encode(shards)
    want = CO.apply(CO.build_matrix(k, m)[k:], shards[:k])
    for r in range(m):
        assert np.array_equal(shards[k + r], want[r]), f"parity {r}"


@pytest.mark.parametrize("k,m", [(200, 56), (128, 128), (1, 255), (255, 1)])
def test_max_shards_encode_and_round_trip(k, m):
    """k + m = 256, klauspost's limit: parity against the oracle, then m
    random erasures (every parity shard lost for 255+1, all but one shard for
    1+255) rebuilt by Reconstruct and ReconstructData."""
    rng = np.random.default_rng(k * 1000 + m)
    s = 1040  # 65 16-B elements: a partial last tile everywhere
    enc = RS.New(k, m)
    full = [rng.integers(0, 256, s, dtype=np.uint8) for _ in range(k)] + [np.zeros(s, np.uint8)
                                                                          for _ in range(m)]
    enc.Encode(full)
    want = CO.apply(CO.build_matrix(k, m)[k:], full[:k])
    for r in range(m):
        assert np.array_equal(full[k + r], want[r]), f"parity {r}"
    missing = set(rng.choice(k + m, size=m, replace=False).tolist())
    sh = [x.copy() if i not in missing else None for i, x in enumerate(full)]
    enc.Reconstruct(sh)
    assert all(np.array_equal(a, b) for a, b in zip(sh, full))
    sh = [x.copy() if i not in missing else None for i, x in enumerate(full)]
    enc.ReconstructData(sh)
    assert all(np.array_equal(sh[i], full[i]) for i in range(k))


@pytest.mark.parametrize("fill", [0x00, 0xFF])
def test_encode_constant_shards(fill):
    enc = RS.New(4, 2)
    shards = [np.full(1024, fill, np.uint8) for _ in range(4)] + [np.zeros(1024, np.uint8) for _ in range(2)]
    enc.Encode(shards)
    want = CO.apply(CO.build_matrix(4, 2)[4:], shards[:4])
    assert all(np.array_equal(shards[4 + r], want[r]) for r in range(2))


def test_encode_ramp():
    enc = RS.New(8, 3)
    ramp = (np.arange(8 * 4096) & 0xFF).astype(np.uint8)
    shards = [ramp[j * 4096:(j + 1) * 4096].copy() for j in range(8)] + [np.zeros(4096, np.uint8)
                                                                       for _ in range(3)]
    enc.Encode(shards)
    want = CO.apply(CO.build_matrix(8, 3)[8:], shards[:8])
    assert all(np.array_equal(shards[8 + r], want[r]) for r in range(3))


@pytest.mark.parametrize("data_only", [False, True])
def test_all_erasure_patterns(vectors, data_only):
    for case in vectors["erasures"]:
        k, m = case["k"], case["m"]
        enc = RS.New(k, m)
        obj = CO.fill_objects(case["index"], 1, case["size"])[0]
        s = case["size"] // k
        full = [obj[j * s:(j + 1) * s].copy() for j in range(k)] + [np.zeros(s, np.uint8) for _ in range(m)]
        enc.Encode(full)
        assert [sha(x) for x in full] == case["shard_sha256"]
        for p in case["patterns"]:
            sh = [x.copy() if i not in p["missing"] else None for i, x in enumerate(full)]
            if data_only:
                enc.ReconstructData(sh)
                for i in range(k + m):
                    if i < k or i not in p["missing"]:
                        assert sha(sh[i]) == case["shard_sha256"][i], (p["missing"], i)
                    else:
                        assert sh[i] is None or len(sh[i]) == 0
            else:
                enc.Reconstruct(sh)
                assert [sha(x) for x in sh] == case["shard_sha256"], p["missing"]


def test_reconstruct_too_many_missing():
    enc = RS.New(4, 2)
    sh = [np.ones(16, np.uint8)] * 3 + [None, None, None]
    with pytest.raises(RS.ErrTooFewShards):
        enc.Reconstruct(sh)


def test_reconstruct_inconsistent_inputs_linear():
    """Reconstruct is a fixed linear map of the first k survivors even for
    inputs that are not a codeword (klauspost semantics, fused parity rows)."""
    rng = np.random.default_rng(5)
    k, m = 4, 2
    sh = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(k + m)]
    for missing in [(0, 5), (1, 4), (3,), (4,), (0, 1)]:
        mine = [x.copy() if i not in missing else None for i, x in enumerate(sh)]
        RS.New(k, m).Reconstruct(mine)
        ref = [x.copy() if i not in missing else np.zeros(0, np.uint8) for i, x in enumerate(sh)]
        O.Encoder(k, m).reconstruct(ref)
        assert all(np.array_equal(a, b) for a, b in zip(mine, ref)), missing


def _split_files(k, m, obj, chunk):
    class W(io.BytesIO):
        pass

    ws = [W() for _ in range(k + m)]
    E.ec_split(k, m, io.BytesIO(obj), chunk, len(obj), ws)
    return [w.getvalue() for w in ws]


def test_ec_split_golden(vectors):
    assert _split_files(3, 2, b"TESTING", 100) == [bytes(f) for f in vectors["testing_3_2"]["files"]]
    for case in vectors["ec_split"]:
        obj = O.object_bytes(case["object_seed_index"], case["size"]).tobytes()
        files = _split_files(case["k"], case["m"], obj, case["chunk"])
        assert [len(f) for f in files] == case["file_len"]
        assert [sha(f) for f in files] == case["file_sha256"], case


def test_ec_split_nil_and_failing_writers():
    obj = O.object_bytes(1, 5000).tobytes()
    want = O.ec_split(4, 2, obj, 1024)

    class Bad:
        def __init__(self):
            self.n = 0

        def write(self, b):
            self.n += 1
            raise IOError("boom")

    ws = [io.BytesIO(), None, Bad(), io.BytesIO(), io.BytesIO(), None]
    E.ec_split(4, 2, io.BytesIO(obj), 1024, len(obj), ws)
    assert ws[0].getvalue() == want[0] and ws[3].getvalue() == want[3] and ws[4].getvalue() == want[4]
    assert ws[2].n == 1  # a failed writer is not written again (ecutils.go:62-68)


@pytest.mark.parametrize("k,m,size,chunk", [(4, 2, 10000, 1024), (4, 2, 7, 100), (8, 3, 100000, 4096),
                                            (4, 2, 3 * MiB + 5, MiB // 4), (3, 2, 1, 100)])
def test_ec_glue_and_reconstruct(k, m, size, chunk):
    obj = O.object_bytes(size + 11, size).tobytes()
    files = _split_files(k, m, obj, chunk)
    assert files == O.ec_split(k, m, obj, chunk)
    for missing in [(), (0,), (k,), (0, k + m - 1), tuple(range(m))]:
        bodies = [None if i in missing else io.BytesIO(f) for i, f in enumerate(files)]
        out = io.BytesIO()
        E.ec_glue(k, m, bodies, chunk, size, out)
        assert out.getvalue() == obj, missing
        if missing:
            bodies = [None if i in missing else io.BytesIO(f) for i, f in enumerate(files)]
            dsts = [io.BytesIO() for _ in missing]
            E.ec_reconstruct(k, m, bodies, chunk, size, dsts, list(missing))
            assert [d.getvalue() for d in dsts] == [files[i] for i in missing]


def test_ec_glue_short_body_is_dropped():
    obj = O.object_bytes(3, 9000).tobytes()
    files = _split_files(4, 2, obj, 1024)
    bodies = [io.BytesIO(f) for f in files]
    bodies[2] = io.BytesIO(files[2][:1500])  # dies in stripe 2
    out = io.BytesIO()
    E.ec_glue(4, 2, bodies, 1024, len(obj), out)
    assert out.getvalue() == obj


# ------------------------------------------------------------------ batches
def _batch(n, k, size, first=0):
    objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, size, first=first)
    return objs


def test_fill_matches_oracle():
    objs = _batch(5, 4, 4096 + 8, first=17)
    want = CO.fill_objects(17, 5, 4096 + 8)
    assert np.array_equal(objs.cpu().numpy(), want)
    odd = torch.zeros((3, 1000), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(odd, 999, first=2)
    got = odd.cpu().numpy()
    assert np.array_equal(got[:, :999], CO.fill_objects(2, 3, 999)) and not got[:, 999].any()


@pytest.mark.parametrize("k,m", [(4, 2), (8, 3)])
@pytest.mark.parametrize("force_stream", [False, True])
def test_batch_encode_1mib_full_compare(k, m, force_stream):
    n, size = 64, MiB
    s = size // k
    objs = _batch(n, k, size, first=100)
    parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    B.set_force_stream(force_stream)
    try:
        B.encode_objects(enc, objs, parity, s)
        torch.cuda.synchronize()
    finally:
        B.set_force_stream(False)
    want, _ = CO.encode_batch(k, m, objs.cpu().numpy(), threads=CO.cpu_threads())
    assert np.array_equal(parity.cpu().numpy(), want)


def test_batch_seeded_vectors(vectors):
    for case in vectors["seeded"]:
        k, m, size = case["k"], case["m"], case["size"]
        s = size // k
        objs = _batch(1, k, size, first=case["index"])
        parity = torch.empty((1, m * s), dtype=torch.uint8, device="cuda")
        B.encode_objects(RS.New(k, m), objs, parity, s)
        o, p = objs.cpu().numpy()[0], parity.cpu().numpy()[0]
        got = [sha(o[j * s:(j + 1) * s]) for j in range(k)] + [sha(p[r * s:(r + 1) * s]) for r in range(m)]
        assert got == case["shard_sha256"]
        assert [list(p[r * s:r * s + 64]) for r in range(m)] == case["parity_head"]


@pytest.mark.parametrize("missing", [(0, 1), (0, 4), (4, 5), (2, 3), (1,), (5,)])
def test_batch_reconstruct_4_2(missing):
    k, m, n, size = 4, 2, 32, MiB
    s = size // k
    objs = _batch(n, k, size, first=9)
    parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    B.encode_objects(enc, objs, parity, s)
    # damaged copy: missing shards overwritten with junk, then rebuilt in place
    objs2, parity2 = objs.clone(), parity.clone()
    views = B.shard_views(objs2, k, s) + B.shard_views(parity2, m, s)
    for i in missing:
        t, col = (objs2, i) if i < k else (parity2, i - k)
        t[:, col * s:(col + 1) * s] = 0xA5
    present = [0 if i in missing else 1 for i in range(k + m)]
    B.reconstruct_views(enc, views, present, n, s)
    torch.cuda.synchronize()
    assert torch.equal(objs2, objs) and torch.equal(parity2, parity)


def test_batch_reconstruct_data_only_keeps_parity():
    k, m, n, size = 8, 3, 16, 4096
    s = size // k
    objs = _batch(n, k, size, first=3)
    parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    B.encode_objects(enc, objs, parity, s)
    objs2, parity2 = objs.clone(), parity.clone()
    objs2[:, :s] = 0
    parity2[:, s:2 * s] = 7
    views = B.shard_views(objs2, k, s) + B.shard_views(parity2, m, s)
    present = [0] + [1] * 7 + [1, 0, 1]
    B.reconstruct_views(enc, views, present, n, s, data_only=True)
    torch.cuda.synchronize()
    assert torch.equal(objs2, objs)
    assert (parity2[:, s:2 * s] == 7).all()


def test_batch_unaligned_views_use_byte_path():
    k, m, n, s = 4, 2, 10, 1001  # odd shard length, unaligned bases
    objs = torch.empty((n, k * s + 3), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s + 3, first=1)
    parity = torch.zeros((n, m * s + 1), dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    base = objs.data_ptr() + 3
    views = [(base + j * s, objs.stride(0)) for j in range(k)]
    views += [(parity.data_ptr() + 1 + r * s, parity.stride(0)) for r in range(m)]
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    o = objs.cpu().numpy()[:, 3:]
    want, _ = CO.encode_batch(k, m, np.ascontiguousarray(o[:, :k * s]))
    p = parity.cpu().numpy()
    assert np.array_equal(p[:, 1:], want)
    assert not p[:, 0].any()


def test_batch_empty_is_noop():
    enc = RS.New(4, 2)
    B.encode_views(enc, [(0x1000, 0)] * 6, 0, 1024)
    B.encode_views(enc, [(0x1000, 0)] * 6, 5, 0)


def test_batch_mixed_sizes_8_3():
    """Config 4 shapes: 4 KiB and 1 MiB objects, 8+3, encode + reconstruct {0,1,2}."""
    k, m = 8, 3
    enc = RS.New(k, m)
    for size, n in [(4096, 256), (MiB, 8)]:
        s = size // k
        objs = _batch(n, k, size, first=size)
        parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
        B.encode_objects(enc, objs, parity, s)
        want, _ = CO.encode_batch(k, m, objs.cpu().numpy(), threads=CO.cpu_threads())
        assert np.array_equal(parity.cpu().numpy(), want)
        objs2 = objs.clone()
        objs2[:, :3 * s] = 0
        views = B.shard_views(objs2, k, s) + B.shard_views(parity, m, s)
        B.reconstruct_views(enc, views, [0, 0, 0] + [1] * 8, n, s)
        torch.cuda.synchronize()
        assert torch.equal(objs2, objs)


def _apply_cases():
    rng = np.random.default_rng(20261016)
    for _ in range(60):
        yield (int(rng.choice([1, 2, 3, 4, 5, 9])), int(rng.choice([1, 3, 4, 8, 9, 16, 17, 33])),
               int(rng.choice([16, 48, 512, 1000, 1024, 4112, 65536])), int(rng.choice([1, 37])))


@pytest.mark.parametrize("rows,cols,s,n", list(_apply_cases()))
def test_apply_random_shapes_match_oracle(rows, cols, s, n):
    """hbec_apply_batch (the general matrix apply under Encode / Reconstruct)
    over random shapes: every kernel family (packed, pipelined, vec, streaming,
    bytes for odd lengths, multi-pass accumulate above 16 inputs / 4 outputs)
    against the oracle, with coefficients 0 and 1 over-represented."""
    rng = np.random.default_rng(rows * 1000 + cols * 10 + s + n)
    coeffs = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    special = rng.random((rows, cols))
    coeffs[special < 0.15] = 0
    coeffs[(special >= 0.15) & (special < 0.3)] = 1
    pad = 32 if s % 16 == 0 else 0  # strided views: row longer than the shards
    ins = torch.from_numpy(rng.integers(0, 256, (n, cols * s + pad), dtype=np.uint8)).cuda()
    outs = torch.full((n, rows * s + pad), 0xA5, dtype=torch.uint8, device="cuda")
    iv = [(ins.data_ptr() + c * s, ins.stride(0)) for c in range(cols)]
    ov = [(outs.data_ptr() + r * s, outs.stride(0)) for r in range(rows)]
    B.apply_views(rows, cols, coeffs.tolist(), iv, ov, n, s)
    torch.cuda.synchronize()
    i_np, o_np = ins.cpu().numpy(), outs.cpu().numpy()
    for o in range(n):
        want = CO.apply(coeffs, [np.ascontiguousarray(i_np[o, c * s:(c + 1) * s]) for c in range(cols)])
        for r in range(rows):
            assert np.array_equal(o_np[o, r * s:(r + 1) * s], want[r]), (o, r)
    assert (o_np[:, rows * s:] == 0xA5).all()


def _reconstruct_cases():
    rng = np.random.default_rng(777)
    for _ in range(40):
        k = int(rng.choice([1, 2, 3, 4, 5, 8, 10, 12, 17, 32]))
        m = int(rng.choice([1, 2, 3, 4, 6, 8]))
        yield k, m, int(rng.choice([16, 512, 1008, 1024, 4096, 65536, 1000, 333])), int(rng.choice([1, 5, 64]))


@pytest.mark.parametrize("k,m,s,n", list(_reconstruct_cases()))
def test_batch_reconstruct_random_erasures(k, m, s, n):
    """Device-batch Encode then Reconstruct / ReconstructData of a random
    erasure set (1..m shards, data and parity mixed) over random shapes:
    rebuilt shards equal the originals; with data_only the erased parity
    slots are left untouched (klauspost ReconstructData)."""
    rng = np.random.default_rng(k * 100 + m * 10 + s + n)
    enc = RS.New(k, m)
    data = torch.from_numpy(rng.integers(0, 256, (n, k * s), dtype=np.uint8)).cuda()
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    views = [(data.data_ptr() + j * s, data.stride(0)) for j in range(k)]
    views += [(par.data_ptr() + r * s, par.stride(0)) for r in range(m)]
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    want = CO.apply(CO.build_matrix(k, m)[k:], [np.ascontiguousarray(data[0, j * s:(j + 1) * s].cpu().numpy())
                                                for j in range(k)])
    assert all(np.array_equal(par[0, r * s:(r + 1) * s].cpu().numpy(), want[r]) for r in range(m))
    n_lost = int(rng.integers(1, m + 1))
    lost = sorted(rng.choice(k + m, size=n_lost, replace=False).tolist())
    for data_only in (False, True):
        d2, p2 = data.clone(), par.clone()
        for i in lost:
            (d2[:, i * s:(i + 1) * s] if i < k else p2[:, (i - k) * s:(i - k + 1) * s]).fill_(0x3C)
        v2 = [(d2.data_ptr() + j * s, d2.stride(0)) for j in range(k)]
        v2 += [(p2.data_ptr() + r * s, p2.stride(0)) for r in range(m)]
        B.reconstruct_views(enc, v2, [0 if i in lost else 1 for i in range(k + m)], n, s, data_only=data_only)
        torch.cuda.synchronize()
        assert torch.equal(d2, data), (lost, data_only)
        if data_only:
            for i in lost:
                if i >= k:
                    assert bool((p2[:, (i - k) * s:(i - k + 1) * s] == 0x3C).all()), i
        else:
            assert torch.equal(p2, par), lost


def test_apply_many_inputs_outputs():
    rng = np.random.default_rng(1)
    rows, cols, n, s = 6, 19, 3, 4096
    coeffs = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    ins = torch.from_numpy(rng.integers(0, 256, (n, cols * s), dtype=np.uint8)).cuda()
    outs = torch.empty((n, rows * s), dtype=torch.uint8, device="cuda")
    B.apply_views(rows, cols, coeffs.tolist(), B.shard_views(ins, cols, s), B.shard_views(outs, rows, s), n, s)
    torch.cuda.synchronize()
    i_np, o_np = ins.cpu().numpy(), outs.cpu().numpy()
    for o in range(n):
        want = CO.apply(coeffs, [i_np[o, c * s:(c + 1) * s] for c in range(cols)])
        assert all(np.array_equal(o_np[o, r * s:(r + 1) * s], want[r]) for r in range(rows))


@pytest.mark.slow
def test_baseline_size_4096x1mib_roundtrip():
    """BASELINE configs[1] + configs[2] at full size: 4096 x 1 MiB, 4+2
    encode, then reconstruct {0,1} into a separate array.  EVERY object's
    parity equals the CPU oracle's (klauspost restatement) and every rebuilt
    shard equals the original data: no sampling."""
    import fullcheck

    k, m, n = 4, 2, 4096
    s = MiB // k
    objs = _batch(n, k, MiB)
    parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    B.encode_objects(enc, objs, parity, s)
    rebuilt = torch.full((n, 2 * s), 0x3C, dtype=torch.uint8, device="cuda")
    views = [(rebuilt.data_ptr(), rebuilt.stride(0)), (rebuilt.data_ptr() + s, rebuilt.stride(0))]
    views += B.shard_views(objs, k, s)[2:] + B.shard_views(parity, m, s)
    B.reconstruct_views(enc, views, [0, 0, 1, 1, 1, 1], n, s)
    torch.cuda.synchronize()
    assert fullcheck.rows_match(rebuilt, objs[:, :2 * s])
    assert fullcheck.encode_parity_matches(k, m, objs, parity) == n


@pytest.mark.parametrize("k,m,s,n", [(4, 2, 5 * 4096 + 48, 7), (8, 3, 3 * 2048 + 16, 5), (2, 2, 4096 * 2 + 1024, 3),
                                     (4, 2, 4096, 1), (6, 3, 16 * 1024, 300), (4, 1, 256 * 1024, 9),
                                     (3, 3, 3 * 1024 + 32, 5), (1, 2, 4 * 4096 + 16, 4), (4, 3, 9 * 1024 + 16, 6)])
def test_batch_pipelined_partial_tiles(k, m, s, n):
    """Shard lengths that are not a multiple of the pipelined kernel's tile,
    and grids with fewer tiles than waves."""
    objs = torch.empty((n, k * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s, first=s)
    parity = torch.full((n, m * s + 64), 0x5A, dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    B.encode_views(enc, B.shard_views(objs, k, s) + [(parity.data_ptr() + r * s, parity.stride(0))
                                                     for r in range(m)], n, s)
    torch.cuda.synchronize()
    want, _ = CO.encode_batch(k, m, objs.cpu().numpy(), threads=CO.cpu_threads())
    got = parity.cpu().numpy()
    assert np.array_equal(got[:, :m * s], want)
    assert (got[:, m * s:] == 0x5A).all()  # nothing written past the last shard
    info = B.kernel_info(k, m, s)
    assert info["tile_bytes"] > 0


# ------------------------------------------------------------------ stripe plans
def _stripe_pool(k, m, sizes, align=16, misalign=()):
    """Host pool of ecSplit databufs: stripe i = object i (k*S data bytes, zero
    padded) followed by m*S parity bytes.  Returns (pool, [(offset, S)])."""
    layout, off = [], 0
    for i, size in enumerate(sizes):
        s = O.ec_shard_length(size, k)
        off = (off + align - 1) // align * align + (3 if i in misalign else 0)
        layout.append((off, s, size))
        off += (k + m) * s
    pool = np.zeros(off + 64, dtype=np.uint8)
    for i, (o, s, size) in enumerate(layout):
        pool[o:o + size] = CO.fill_objects(1000 + i, 1, size)[0]
    return pool, layout


def _expected_pool(k, m, pool, layout):
    want = pool.copy()
    mat = CO.build_matrix(k, m)[k:]
    for o, s, _ in layout:
        data = [want[o + j * s:o + (j + 1) * s] for j in range(k)]
        for r, p in enumerate(CO.apply(mat, data)):
            want[o + (k + r) * s:o + (k + r + 1) * s] = p
    return want


@pytest.mark.parametrize("k,m,sizes,misalign", [
    (8, 3, [4096, MiB, 4096, 4096, MiB, 4096, MiB, 4096] * 3, ()),
    (4, 2, [MiB, 7, 4096, 1001, MiB + 16, 64, 4097], (1, 3)),
    (10, 4, [4096, 40960, 160], ()),
    (5, 5, [5 * 4096, 5 * 100000, 80], ()),
    # near-uniform odd sizes: per-object records (gf_odd_planrec + gf_odd_rec)
    (12, 4, [MiB - i for i in range(1, 9)], (2, 5)),
    (8, 3, [MiB - 8 * i - 3 for i in range(6)], (0,)),
    (4, 2, [MiB - 4, MiB - 3, MiB - 1, MiB - 2], (1,)),
    (20, 4, [20 * 5000 + 1 + i for i in range(5)], (3,)),
])
def test_plan_encode_reconstruct_mixed(k, m, sizes, misalign):
    pool, layout = _stripe_pool(k, m, sizes, misalign=misalign)
    want = _expected_pool(k, m, pool, layout)
    dev = torch.from_numpy(pool).cuda()
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, [(dev.data_ptr() + o, s) for o, s, _ in layout])
    info = plan.info()
    assert info["shard_bytes"] == sum(s for _, s, _ in layout)
    plan.encode()
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), want)
    # erase up to m shards of every stripe (data first), rebuild in place
    for missing in [tuple(range(min(m, 3))), (0, k), (k - 1,), tuple(range(k, k + m))]:
        damaged = torch.from_numpy(want.copy()).cuda()
        for o, s, _ in layout:
            for i in missing:
                damaged[o + i * s:o + (i + 1) * s] = 0xEE
        dplan = B.StripePlan(enc, [(damaged.data_ptr() + o, s) for o, s, _ in layout])
        dplan.reconstruct([0 if i in missing else 1 for i in range(k + m)])
        torch.cuda.synchronize()
        assert np.array_equal(damaged.cpu().numpy(), want), missing


def test_plan_config4_shape_counts():
    """Config 4 plan: 8+3, 4 KiB and 1 MiB objects drawn p=0.5 by splitmix64."""
    k, m = 8, 3
    flags = O.splitmix_bytes(O.HBEC_SEED, 64)
    sizes = [MiB if b & 1 else 4096 for b in flags]
    pool, layout = _stripe_pool(k, m, sizes)
    dev = torch.from_numpy(pool).cuda()
    plan = B.StripePlan(RS.New(k, m), [(dev.data_ptr() + o, s) for o, s, _ in layout])
    info = plan.info()
    tile = info["tile_bytes"]
    assert info["n_tiles"] == sum((s + tile - 1) // tile for _, s, _ in layout)
    assert info["n_fallback"] == sum(R.stripe_on_records(k, m, dev.data_ptr() + o, s) for o, s, _ in layout)
    plan.encode()
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), _expected_pool(k, m, pool, layout))


def _object_arenas(k, m, sizes, misalign=()):
    """Object-plan layout: objects back to back in a data arena (k*S bytes
    each, zero padded), their parity back to back in a parity arena."""
    dl, pl, doff, poff = [], [], 0, 0
    for i, size in enumerate(sizes):
        s = O.ec_shard_length(size, k)
        doff = (doff + 15) // 16 * 16 + (5 if i in misalign else 0)
        poff = (poff + 15) // 16 * 16
        dl.append((doff, s, size))
        pl.append(poff)
        doff += k * s
        poff += m * s
    data = np.zeros(doff + 64, dtype=np.uint8)
    for i, (o, s, size) in enumerate(dl):
        data[o:o + size] = CO.fill_objects(2000 + i, 1, size)[0]
    parity = np.zeros(poff + 64, dtype=np.uint8)
    mat = CO.build_matrix(k, m)[k:]
    for (o, s, _), po in zip(dl, pl):
        for r, par in enumerate(CO.apply(mat, [data[o + j * s:o + (j + 1) * s] for j in range(k)])):
            parity[po + r * s:po + (r + 1) * s] = par
    return data, parity, dl, pl


@pytest.mark.parametrize("k,m,sizes,misalign", [
    (8, 3, [4096, MiB, 4096, 4096, MiB, 4096, MiB, 4096] * 3, ()),
    (4, 2, [MiB, 7, 4096, 1001, MiB + 16, 64, 4097], (1, 3)),
    (10, 4, [4096, 40960, 160], ()),
    (5, 5, [5 * 4096, 5 * 100000, 80], ()),
    # near-uniform odd sizes: per-object records (gf_odd_planrec + gf_odd_rec)
    (12, 4, [MiB - i for i in range(1, 9)], (2, 5)),
    (8, 3, [MiB - 8 * i - 3 for i in range(6)], (0,)),
    (4, 2, [MiB - 4, MiB - 3, MiB - 1, MiB - 2], (1,)),
    (20, 4, [20 * 5000 + 1 + i for i in range(5)], (3,)),
])
def test_object_plan_encode_reconstruct(k, m, sizes, misalign):
    """hbec_plan_objects: data and parity in separate arenas; every erasure
    pattern family rebuilds into the right arena."""
    data, parity, dl, pl = _object_arenas(k, m, sizes, misalign)
    enc = RS.New(k, m)
    d = torch.from_numpy(data).cuda()
    p = torch.zeros(parity.size, dtype=torch.uint8, device="cuda")

    def objs(dt, pt):
        return [(dt.data_ptr() + o, pt.data_ptr() + po, s) for (o, s, _), po in zip(dl, pl)]

    plan = B.StripePlan(enc, objects=objs(d, p))
    assert plan.info()["n_fallback"] == sum(R.object_on_records(k, m, d.data_ptr() + o, p.data_ptr() + po, s)
                                            for (o, s, _), po in zip(dl, pl))
    plan.encode()
    torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy(), parity)
    assert np.array_equal(d.cpu().numpy(), data)
    for missing in [tuple(range(min(m, 3))), (0, k), (k - 1,), tuple(range(k, k + m)), (k - 1, k + m - 1)]:
        dd = torch.from_numpy(data.copy()).cuda()
        pp = torch.from_numpy(parity.copy()).cuda()
        for (o, s, _), po in zip(dl, pl):
            for i in missing:
                if i < k:
                    dd[o + i * s:o + (i + 1) * s] = 0xEE
                else:
                    pp[po + (i - k) * s:po + (i - k + 1) * s] = 0xEE
        B.StripePlan(enc, objects=objs(dd, pp)).reconstruct([0 if i in missing else 1 for i in range(k + m)])
        torch.cuda.synchronize()
        assert np.array_equal(dd.cpu().numpy(), data), missing
        assert np.array_equal(pp.cpu().numpy(), parity), missing


def test_plan_empty_and_zero_length():
    enc = RS.New(4, 2)
    B.StripePlan(enc, []).encode()
    B.StripePlan(enc, [(0x1000, 0)]).encode()
    torch.cuda.synchronize()


def test_plan_rejects_other_codec_shape():
    buf = torch.zeros(6 * 4096, dtype=torch.uint8, device="cuda")
    plan = B.StripePlan(RS.New(4, 2), [(buf.data_ptr(), 4096)])
    with pytest.raises(RS.ErrInvalidArg):
        N_plan_encode = __import__("hummingbird_amd._native", fromlist=["lib"]).lib().hbec_encode_plan
        RS.check(N_plan_encode(RS.New(8, 3).handle, plan._h, None))


# ------------------------------------------------------------ streaming host path
def _host_stripes(k, m, sizes, seed=0):
    stripes = []
    for i, size in enumerate(sizes):
        s = O.ec_shard_length(size, k)
        st = np.zeros((k + m) * s, dtype=np.uint8)
        st[:size] = CO.fill_objects(seed + i, 1, size)[0]
        stripes.append(st)
    return stripes


def _encoded_copy(k, m, stripes):
    mat = CO.build_matrix(k, m)[k:]
    out = []
    for st in stripes:
        s = st.size // (k + m)
        w = st.copy()
        for r, p in enumerate(CO.apply(mat, [w[j * s:(j + 1) * s] for j in range(k)])):
            w[(k + r) * s:(k + r + 1) * s] = p
        out.append(w)
    return out


@pytest.mark.parametrize("k,m,sizes", [
    (4, 2, [MiB] * 70 + [7, 4096, 1001]),          # > one 64 MiB slot of 1 MiB objects
    (8, 3, [4096, MiB, 4096, 3 * MiB + 8, 1]),
    (4, 2, [68 * MiB]),                             # one stripe wider than a slot (column pieces)
    (3, 5, [3000, 30000]),                          # more outputs than inputs, 2 row groups
])
def test_host_path_encode_reconstruct(k, m, sizes):
    enc = RS.New(k, m)
    stripes = _host_stripes(k, m, sizes, seed=len(sizes))
    want = _encoded_copy(k, m, stripes)
    enc.EncodeStripes(stripes)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    for missing in [tuple(range(min(m, 3))), (0, k)]:
        damaged = [w.copy() for w in want]
        for st in damaged:
            s = st.size // (k + m)
            for i in missing:
                st[i * s:(i + 1) * s] = 0x33
        enc.ReconstructStripes(damaged, [0 if i in missing else 1 for i in range(k + m)])
        for got, w in zip(damaged, want):
            assert np.array_equal(got, w), missing


def _pinned_stripes(buf, k, m, sizes, seed, gap=0):
    """Stripes laid out back to back (16-B aligned starts, `gap` bytes apart)
    inside one pinned host buffer's numpy view."""
    out, off = [], 0
    for i, size in enumerate(sizes):
        s = O.ec_shard_length(size, k)
        st = buf[off:off + (k + m) * s]
        st[:] = 0
        st[:size] = CO.fill_objects(seed + i, 1, size)[0]
        out.append(st)
        off = (off + (k + m) * s + gap + 15) // 16 * 16
    return out


@pytest.mark.parametrize("k,m,sizes", [
    (4, 2, [MiB] * 40 + [4096, 1001, 16 * 7]),      # 1001 -> S=251: unaligned, zero-copy via gf_apply_unaligned_plan
    (8, 3, [4096, MiB, 4096, 3 * MiB + 8, 1]),
    (3, 5, [3000 * 16, 30000 * 16]),                # more outputs than inputs, 2 row groups
])
def test_host_path_zero_copy_pinned(k, m, sizes):
    """Stripes in hbec_host_alloc memory are coded in place by the GPU (no
    staging); the batch also mixes in pageable stripes, which take the ring."""
    enc = RS.New(k, m)
    total = sum((k + m) * O.ec_shard_length(x, k) + 16 for x in sizes) + 16
    hb = RS.HostBuffer(total)
    pinned = _pinned_stripes(hb.array, k, m, sizes, seed=3)
    pageable = _host_stripes(k, m, [MiB, 5000], seed=99)
    assert all(RS.host_device_addr(st) != 0 for st in pinned)
    assert all(RS.host_device_addr(st) == 0 for st in pageable)
    stripes = pinned[:len(pinned) // 2] + pageable + pinned[len(pinned) // 2:]
    want = _encoded_copy(k, m, stripes)
    enc.EncodeStripes(stripes)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    for missing in [tuple(range(min(m, 3))), (0, k)]:
        for st in stripes:
            s = st.size // (k + m)
            for i in missing:
                st[i * s:(i + 1) * s] = 0x5A
        enc.ReconstructStripes(stripes, [0 if i in missing else 1 for i in range(k + m)])
        for got, w in zip(stripes, want):
            assert np.array_equal(got, w), missing
    del stripes, pinned
    hb.free()


def _host_random_cases():
    rng = np.random.default_rng(4242)
    for _ in range(10):
        k = int(rng.choice([2, 3, 4, 6, 8, 10, 12]))
        m = int(rng.choice([1, 2, 3, 4, 5]))
        sizes = [int(x) for x in rng.choice([1, 17, 4096, 4096 * 3 + 5, 65536, MiB, MiB + 48, 5 * MiB], size=9)]
        yield k, m, sizes


@pytest.mark.parametrize("k,m,sizes", list(_host_random_cases()))
def test_host_path_random_mixed(k, m, sizes):
    """Random shapes through the host path: pinned stripes (zero-copy when
    aligned) interleaved with pageable ones (staging ring), encoded against
    the oracle, then a random erasure set rebuilt."""
    rng = np.random.default_rng(k * 31 + m + len(sizes))
    enc = RS.New(k, m)
    half = sizes[: len(sizes) // 2]
    total = sum((k + m) * O.ec_shard_length(x, k) + 16 for x in half) + 16
    hb = RS.HostBuffer(total)
    pinned = _pinned_stripes(hb.array, k, m, half, seed=k + m)
    pageable = _host_stripes(k, m, sizes[len(sizes) // 2:], seed=7 * k + m)
    stripes = [x for pair in zip(pinned, pageable) for x in pair] + pageable[len(pinned):]
    want = _encoded_copy(k, m, stripes)
    enc.EncodeStripes(stripes)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    lost = sorted(rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False).tolist())
    for st in stripes:
        sl = st.size // (k + m)
        for i in lost:
            st[i * sl:(i + 1) * sl] = 0x6B
    enc.ReconstructStripes(stripes, [0 if i in lost else 1 for i in range(k + m)])
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w), lost
    del stripes, pinned
    hb.free()


def test_host_path_zero_copy_foreign_pinned_memory():
    """Pinned memory the library did not allocate (torch pin_memory ->
    hipHostMalloc) is recognised through the runtime's pointer attributes."""
    k, m, S, n = 4, 2, MiB // 4, 64
    host = torch.zeros((n, (k + m) * S), dtype=torch.uint8).pin_memory()
    arr = host.numpy()
    objs = CO.fill_objects(7, n, k * S)
    arr[:, :k * S] = objs
    rows = [arr[i] for i in range(n)]
    assert RS.host_device_addr(rows[0]) != 0
    enc = RS.New(k, m)
    enc.EncodeStripes(rows)
    want, _ = CO.encode_batch(k, m, objs, threads=CO.cpu_threads())
    assert np.array_equal(arr[:, k * S:], want)
    arr[:, :2 * S] = 0
    enc.ReconstructStripes(rows, [0, 0, 1, 1, 1, 1])
    assert np.array_equal(arr[:, :k * S], objs)


@pytest.mark.parametrize("k,m,s", [(4, 2, MiB // 4), (8, 3, 4096), (3, 2, 48), (4, 2, 1001)])
def test_per_call_encode_reconstruct_zero_copy(k, m, s):
    """klauspost Encode / Reconstruct on shards that live in pinned host memory:
    coded in place by the GPU (no staging); S % 16 != 0 (1001) through the
    unaligned kernel."""
    hb = RS.HostBuffer((k + m) * (s + 16) + 16)
    pitch = (s + 15) // 16 * 16
    shards = [hb.array[i * pitch:i * pitch + s] for i in range(k + m)]
    data = CO.fill_objects(5, 1, k * s)[0]
    for j in range(k):
        shards[j][:] = data[j * s:(j + 1) * s]
    enc = RS.New(k, m)
    enc.Encode(shards)
    want = CO.apply(CO.build_matrix(k, m)[k:], [data[j * s:(j + 1) * s] for j in range(k)])
    for r in range(m):
        assert np.array_equal(shards[k + r], want[r])
    # rebuild data shard 0 and parity shard 0 into their pinned slots (cap >= S)
    keep = [x.copy() for x in shards]
    shards[0][:] = 0
    shards[k][:] = 0
    enc.Reconstruct([None if i in (0, k) else shards[i] for i in range(k + m)])  # fresh arrays
    enc.Reconstruct([shards[i][:0] if i in (0, k) else shards[i] for i in range(k + m)])  # reuse capacity
    del shards
    hb.free()
    assert all(np.array_equal(a, b) for a, b in zip(keep[1:k], keep[1:k]))


def test_host_alloc_errors_and_ranges():
    with pytest.raises(RS.ErrInvalidArg):
        RS.HostBuffer(0)
    hb = RS.HostBuffer(4096)
    assert RS.host_device_addr(hb.array[16:4096]) == RS.host_device_addr(hb.array) + 16
    hb.free()
    hb.free()  # idempotent


@pytest.mark.parametrize("devices", [None, [0], [0, 0], [0, 0, 0]])
def test_host_path_devices_partition(devices):
    """hbec_*_host_devices: stripes cut into per-device runs coded by one host
    thread each (here several threads share device 0, each with its own ring),
    pageable and pinned stripes mixed."""
    k, m = 4, 2
    sizes = [MiB] * 9 + [4096, 1001, 3 * MiB + 8, 7]
    enc = RS.New(k, m)
    hb = RS.HostBuffer(sum((k + m) * O.ec_shard_length(x, k) + 16 for x in sizes[:6]) + 16)
    stripes = _pinned_stripes(hb.array, k, m, sizes[:6], seed=11) + _host_stripes(k, m, sizes[6:], seed=17)
    want = _encoded_copy(k, m, stripes)
    enc.EncodeStripesDevices(stripes, devices)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    missing = (1, k)
    for st in stripes:
        sl = st.size // (k + m)
        for i in missing:
            st[i * sl:(i + 1) * sl] = 0x77
    enc.ReconstructStripesDevices(stripes, [0 if i in missing else 1 for i in range(k + m)], devices=devices)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    del stripes
    hb.free()


def test_host_path_devices_errors():
    enc = RS.New(4, 2)
    st = _host_stripes(4, 2, [4096])
    with pytest.raises(RS.ReedSolomonError):
        enc.EncodeStripesDevices(st, devices=[RS.device_count() + 3])
    assert RS.device_count() >= 1
    enc.EncodeStripesDevices([], devices=[0])


# k > 8 (a `hec` policy may set any data_shards, ecengine.go:719-724): the
# stripes kernel runs in passes of <= 8 inputs, later passes accumulating.
WIDE = [(10, 4, [MiB, 4096 * 10, 1000, MiB + 160, 16 * 10]), (17, 3, [17 * 4096, 17 * 1024 * 3 + 17 * 16, 5]),
        (12, 5, [12 * 8192, 12 * 16])]


def _wide_patterns(k, m):
    return [tuple(range(min(m, 3))), (0, k), (k - 1, 8, 9)[:m], tuple(range(k - m, k))]


@pytest.mark.parametrize("k,m,sizes", WIDE)
def test_host_path_wide_k_ring(k, m, sizes):
    enc = RS.New(k, m)
    stripes = _host_stripes(k, m, sizes, seed=k * 3 + m)
    want = _encoded_copy(k, m, stripes)
    enc.EncodeStripes(stripes)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    for missing in _wide_patterns(k, m):
        damaged = [w.copy() for w in want]
        for st in damaged:
            s = st.size // (k + m)
            for i in missing:
                st[i * s:(i + 1) * s] = 0x3C
        enc.ReconstructStripes(damaged, [0 if i in missing else 1 for i in range(k + m)])
        for got, w in zip(damaged, want):
            assert np.array_equal(got, w), missing


@pytest.mark.parametrize("k,m,sizes", WIDE)
def test_host_path_wide_k_zero_copy(k, m, sizes):
    enc = RS.New(k, m)
    total = sum((k + m) * O.ec_shard_length(x, k) + 16 for x in sizes) + 16
    hb = RS.HostBuffer(total)
    stripes = _pinned_stripes(hb.array, k, m, sizes, seed=5 * k + m)
    want = _encoded_copy(k, m, stripes)
    enc.EncodeStripes(stripes)
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    missing = _wide_patterns(k, m)[1]
    for st in stripes:
        s = st.size // (k + m)
        for i in missing:
            st[i * s:(i + 1) * s] = 0xC3
    enc.ReconstructStripes(stripes, [0 if i in missing else 1 for i in range(k + m)])
    for got, w in zip(stripes, want):
        assert np.array_equal(got, w)
    del stripes
    hb.free()


@pytest.mark.parametrize("k,m", [(10, 4), (17, 3)])
def test_batcher_wide_k(k, m):
    import threading

    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=64 << 20, max_wait_us=1000)
    sizes = [k * 4096 * (1 + i % 5) for i in range(24)]
    stripes = _host_stripes(k, m, sizes, seed=k + 100)
    want = _encoded_copy(k, m, stripes)
    errors = []

    def run(i):
        try:
            bat.Encode(stripes[i])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    threads = [threading.Thread(target=run, args=(i,)) for i in range(len(stripes))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    bat.close()
    assert not errors
    assert all(np.array_equal(a, b) for a, b in zip(stripes, want))


@pytest.mark.parametrize("k,m", [(10, 4), (17, 3)])
def test_stripe_plan_wide_k(k, m):
    """Stripe plans with k > 8: the tiled kernel in accumulate passes, except
    the stripes the record kernels take (10+4 with S >= 24 KiB, rec_route)."""
    sizes = [k * 1024 * 3, k * 16, MiB // 4 * k, k * 4096]
    pool, layout = _stripe_pool(k, m, sizes)
    want = _expected_pool(k, m, pool, layout)
    dev = torch.from_numpy(pool).cuda()
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, [(dev.data_ptr() + o, s) for o, s, _ in layout])
    assert plan.info()["n_fallback"] == sum(R.stripe_on_records(k, m, dev.data_ptr() + o, s) for o, s, _ in layout)
    plan.encode()
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), want)
    for missing in [(0, 3, k)[:m], (k - 1, 8, 9)[:m]]:
        damaged = torch.from_numpy(want.copy()).cuda()
        for o, s, _ in layout:
            for i in missing:
                damaged[o + i * s:o + (i + 1) * s] = 0xEE
        dplan = B.StripePlan(enc, [(damaged.data_ptr() + o, s) for o, s, _ in layout])
        dplan.reconstruct([0 if i in missing else 1 for i in range(k + m)])
        torch.cuda.synchronize()
        assert np.array_equal(damaged.cpu().numpy(), want), missing


# ------------------------------------------------------------------ Verify
@pytest.mark.parametrize("k,m,n", [(4, 2, 4096), (8, 3, 1000), (5, 5, 17), (10, 4, 3000), (2, 1, 1)])
def test_verify_host(k, m, n):
    enc = RS.New(k, m)
    rng = np.random.default_rng(k + m + n)
    shards = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(m)]
    assert enc.Verify(shards) is (m == 0)
    enc.Encode(shards)
    assert enc.Verify(shards)
    for victim in (0, k - 1, k, k + m - 1):
        bad = [s.copy() for s in shards]
        bad[victim][n // 2] ^= 0x40
        assert not enc.Verify(bad), victim
    with pytest.raises(RS.ErrShardSize):
        enc.Verify(shards[:-1] + [np.zeros(n + 1, np.uint8)])
    with pytest.raises(RS.ErrTooFewShards):
        enc.Verify(shards[:-1])


@pytest.mark.parametrize("k,m,size,unaligned", [(4, 2, MiB, False), (8, 3, 4096, False), (8, 3, MiB, False),
                                                (4, 2, 1000 * 4, True), (12, 4, 12 * 4096, False)])
def test_verify_batch_flags(k, m, size, unaligned):
    n = 64
    s = size // k
    extra = 3 if unaligned else 0
    objs = torch.empty((n, k * s + extra), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s + extra)
    parity = torch.empty((n, m * s + extra), dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    views = [(objs.data_ptr() + extra + j * s, objs.stride(0)) for j in range(k)]
    views += [(parity.data_ptr() + extra + r * s, parity.stride(0)) for r in range(m)]
    B.encode_views(enc, views, n, s)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.sum()) == 0
    corrupt = {3: ("data", 0, 5), 17: ("parity", m - 1, s - 1), 40: ("data", k - 1, s // 2), 63: ("parity", 0, 0)}
    for o, (kind, i, off) in corrupt.items():
        t = objs if kind == "data" else parity
        t[o, extra + i * s + off] ^= 0x01
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert sorted(torch.nonzero(flags).flatten().tolist()) == sorted(corrupt)


# ------------------------------------------------------------ batching driver
def test_batcher_concurrent_callers_share_launches():
    import threading

    k, m = 4, 2
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=64 << 20, max_wait_us=2000)
    sizes = [MiB if i % 3 else 4096 + 16 * i for i in range(48)]
    stripes = _host_stripes(k, m, sizes, seed=77)
    want = _encoded_copy(k, m, stripes)
    errors = []

    def worker(idx):
        try:
            bat.Encode(stripes[idx])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(len(stripes))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors
    assert all(np.array_equal(a, b) for a, b in zip(stripes, want))
    st = bat.stats()
    assert st["stripes"] == len(stripes) and st["batches"] < len(stripes)
    # reconstruct through the batcher too
    damaged = [w.copy() for w in want]
    for d in damaged:
        s = d.size // (k + m)
        d[:s] = 0
    threads = [threading.Thread(target=lambda i=i: bat.Reconstruct(damaged[i], [0, 1, 1, 1, 1, 1]))
               for i in range(len(damaged))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert all(np.array_equal(a, b) for a, b in zip(damaged, want))
    bat.close()


@pytest.mark.parametrize("workers", ["1", "3"])
def test_batcher_mixed_ops_and_patterns_concurrently(monkeypatch, workers):
    """Encodes and reconstructs with three erasure patterns (data-only and
    full) in flight at once: every batch must be one homogeneous group, and
    every caller must get exactly its own result, whatever the worker count."""
    import threading

    monkeypatch.setenv("HBEC_BATCHER_WORKERS", workers)
    k, m = 4, 2
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=24 << 20, max_wait_us=500)
    sizes = [MiB if i % 4 else 4096 + 16 * i for i in range(60)]
    stripes = _host_stripes(k, m, sizes, seed=91)
    want = _encoded_copy(k, m, stripes)
    patterns = [([0, 1, 1, 1, 1, 1], False), ([1, 1, 0, 1, 0, 1], False), ([0, 1, 1, 0, 1, 1], True)]
    jobs = []
    for i, w in enumerate(want):
        if i % 4 == 0:
            jobs.append(("enc", stripes[i], None, False))
            continue
        present, data_only = patterns[i % 3]
        d = w.copy()
        s = d.size // (k + m)
        for j, p in enumerate(present):
            if not p:
                d[j * s:(j + 1) * s] = 0
        jobs.append(("rec", d, present, data_only))
    errors = []

    def run(job):
        op, buf, present, data_only = job
        try:
            if op == "enc":
                bat.Encode(buf)
            else:
                bat.Reconstruct(buf, present, data_only=data_only)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    threads = [threading.Thread(target=run, args=(j,)) for j in jobs]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors
    for (op, buf, present, data_only), w in zip(jobs, want):
        if op == "enc" or not data_only:
            assert np.array_equal(buf, w)
        else:  # data-only: the data shards are rebuilt, missing parity stays as it was (zeroed)
            s = w.size // (k + m)
            assert np.array_equal(buf[:k * s], w[:k * s])
    st = bat.stats()
    assert st["stripes"] == len(jobs)
    bat.close()


def test_batcher_bad_request_fails_alone():
    """A caller's invalid stripe (null base; an MD5 stripe wider than a
    staging slot) is rejected at submit and never fails the callers it
    would have been batched with; a reconstruct queued between encodes does
    not split the encodes' batch."""
    import ctypes as C
    import threading

    from hummingbird_amd import _native as N

    k, m = 4, 2
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=64 << 20, max_wait_us=3000)
    stripes = _host_stripes(k, m, [4096 * (1 + i % 3) for i in range(24)], seed=5)
    want = _encoded_copy(k, m, stripes)
    damaged = want[0].copy()
    s0 = damaged.size // (k + m)
    damaged[:s0] = 0
    errors, bad_rc = [], []

    def good(i):
        try:
            bat.Encode(stripes[i])
        except Exception as e:  # pragma: no cover
            errors.append(e)

    def bad_null():
        st = N.Stripe()
        st.base = None
        st.shard_len = 4096
        bad_rc.append(N.lib().hbec_batcher_encode(bat._h, C.byref(st)))

    def bad_wide():
        st = N.Stripe()
        st.base = stripes[0].ctypes.data
        st.shard_len = 1 << 40  # never dereferenced: rejected before queueing
        dig = (C.c_uint8 * (16 * (k + m)))()
        bad_rc.append(N.lib().hbec_batcher_encode_md5(bat._h, C.byref(st), dig))

    def rec():
        try:
            bat.Reconstruct(damaged, [0, 1, 1, 1, 1, 1])
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=good, args=(i,)) for i in range(12)] + [threading.Thread(target=bad_null),
                                                                        threading.Thread(target=rec),
                                                                        threading.Thread(target=bad_wide)]
    th += [threading.Thread(target=good, args=(i,)) for i in range(12, 24)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    bat.close()
    assert not errors
    assert sorted(bad_rc) == [N.ERR_INVALID_ARG, N.ERR_INVALID_ARG]
    assert all(np.array_equal(a, b) for a, b in zip(stripes, want))
    assert np.array_equal(damaged, want[0])
