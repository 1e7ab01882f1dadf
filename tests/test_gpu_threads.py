"""Thread safety of the C ABI (SURVEY §8b "Threading": cgo calls arrive on
arbitrary OS threads, so every hbec_* entry point must be safe to call
concurrently).  ctypes drops the GIL around each call, so these Python
threads really overlap inside libhbec: shared codecs (decode-matrix cache,
staging pool), per-thread streams, device batches and MD5 chains at once.
Results are checked against the oracle per call.
"""
import threading

import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from hummingbird_amd import shardhash as H
from oracle import coracle as CO
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _run(workers):
    errs = []

    def wrap(fn, i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append((i, repr(e)))

    ths = [threading.Thread(target=wrap, args=(fn, i)) for i, fn in enumerate(workers)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs


def test_shared_codecs_host_calls_from_many_threads():
    codecs = {(4, 2): RS.New(4, 2), (8, 3): RS.New(8, 3)}
    mats = {km: CO.build_matrix(*km) for km in codecs}

    def worker(t):
        rng = np.random.default_rng(1000 + t)
        k, m = (4, 2) if t % 2 == 0 else (8, 3)
        enc, mat = codecs[(k, m)], mats[(k, m)]
        for _ in range(12):
            n = int(rng.integers(1, 200_000))
            data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
            shards = [d.copy() for d in data] + [np.zeros(n, np.uint8) for _ in range(m)]
            enc.Encode(shards)
            want = CO.apply(mat[k:], data)
            for r in range(m):
                assert np.array_equal(shards[k + r], want[r])
            # random erasure pattern (<= m missing) through the shared decode cache
            miss = sorted(rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False).tolist())
            orig = [s.copy() for s in shards]
            for i in miss:
                shards[i] = np.zeros(0, np.uint8)
            enc.Reconstruct(shards)
            for i in range(k + m):
                assert np.array_equal(shards[i], orig[i]), (t, miss, i)
            assert enc.Verify(shards)

    _run([worker] * 8)


def test_device_batches_and_md5_on_separate_streams():
    k, m, S, n = 4, 2, 64 * 1024, 48
    enc = RS.New(k, m)

    def worker(t):
        torch.cuda.set_device(0)
        stream = torch.cuda.Stream()
        with torch.cuda.stream(stream):
            objs = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(objs, k * S, first=100 * t, stream=stream)
            par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            dig = H.encode_objects_md5(enc, objs, par, S, stream=stream)
            views = B.shard_views(objs, k, S) + B.shard_views(par, m, S)
            rebuilt = torch.empty((n, 2 * S), dtype=torch.uint8, device="cuda")
            rv = list(views)
            rv[0] = (rebuilt.data_ptr(), rebuilt.stride(0))
            rv[4] = (rebuilt.data_ptr() + S, rebuilt.stride(0))
            B.reconstruct_views(enc, rv, [0, 1, 1, 1, 0, 1], n, S, stream=stream)
        stream.synchronize()
        host = objs.cpu().numpy()
        want_par, _ = CO.encode_batch(k, m, host)
        assert np.array_equal(par.cpu().numpy(), want_par)
        assert torch.equal(rebuilt[:, :S], objs[:, :S])
        assert torch.equal(rebuilt[:, S:], par[:, :S])
        got = H.hexdigests(dig)
        for o in (0, n - 1):
            shards = [host[o, j * S:(j + 1) * S] for j in range(k)] + [want_par[o, r * S:(r + 1) * S]
                                                                        for r in range(m)]
            assert got[o] == [O.shard_hash(x) for x in shards]

    _run([worker] * 6)


def test_batcher_and_direct_calls_interleaved():
    k, m, S = 4, 2, 32 * 1024
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=16 << 20, max_wait_us=200)
    mat = CO.build_matrix(k, m)

    def worker(t):
        rng = np.random.default_rng(7 + t)
        for i in range(10):
            stripe = np.zeros((k + m) * S, np.uint8)
            stripe[:k * S] = rng.integers(0, 256, k * S, dtype=np.uint8)
            if (t + i) % 2:
                bat.Encode(stripe)
            else:
                shards = [stripe[j * S:(j + 1) * S] for j in range(k + m)]
                enc.Encode(shards)
            want = CO.apply(mat[k:], [stripe[j * S:(j + 1) * S] for j in range(k)])
            for r in range(m):
                assert np.array_equal(stripe[(k + r) * S:(k + r + 1) * S], want[r])

    try:
        _run([worker] * 8)
    finally:
        bat.close()
