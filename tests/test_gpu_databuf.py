"""Single-pointer databuf entry points (hbec_encode_databuf /
hbec_reconstruct_databuf / hbec_verify_databuf): the k+m shards of ONE
contiguous buffer, shard i at databuf + i*S — the slices every
objectserver/ecutils.go call site hands klauspost (ecSplit :31-35,55-59;
ecReconstruct :94-111; ecGlue :151-168).  Checked byte for byte against the
CPU oracle (oracle/oracle.py, klauspost's default codec restated)."""
import io
import itertools

import numpy as np
import pytest
import torch

from hummingbird_amd import ecutils as E
from hummingbird_amd import reedsolomon as RS
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    yield


def _databuf(k, m, s, seed):
    buf = np.zeros((k + m) * s, dtype=np.uint8)
    buf[:k * s] = O.object_bytes(seed, k * s)
    return buf


def _oracle_encode(k, m, buf, s):
    shards = [buf[i * s:(i + 1) * s].copy() for i in range(k + m)]
    O.Encoder(k, m).encode(shards)
    return np.concatenate(shards)


@pytest.mark.parametrize("k,m,s", [(4, 2, 262144), (8, 3, 512), (8, 3, 131072), (10, 4, 1003), (3, 2, 3),
                                   (17, 3, 4096), (2, 1, 1)])
def test_encode_databuf_matches_oracle(k, m, s):
    enc = RS.New(k, m)
    buf = _databuf(k, m, s, 100 * k + m)
    want = _oracle_encode(k, m, buf, s)
    enc.EncodeDatabuf(buf, s)
    assert np.array_equal(buf, want)
    assert enc.VerifyDatabuf(buf, s)


@pytest.mark.parametrize("k,m,s", [(4, 2, 4096), (8, 3, 512), (10, 4, 1000)])
def test_reconstruct_databuf_every_pattern(k, m, s):
    """Every erasure pattern of <= m shards (<= 2 for 10+4 to bound the run):
    the missing shards are rebuilt IN THEIR SLOTS; ReconstructData rebuilds
    data slots only and leaves missing parity slots untouched."""
    enc = RS.New(k, m)
    full = _oracle_encode(k, m, _databuf(k, m, s, 7 * k + m), s)
    max_e = m if k + m <= 11 else 2
    for e in range(1, max_e + 1):
        for missing in itertools.combinations(range(k + m), e):
            present = [0 if i in missing else 1 for i in range(k + m)]
            buf = full.copy()
            for i in missing:
                buf[i * s:(i + 1) * s] = 0xA5
            enc.ReconstructDatabuf(buf, s, present)
            assert np.array_equal(buf, full), missing
            buf = full.copy()
            for i in missing:
                buf[i * s:(i + 1) * s] = 0xA5
            enc.ReconstructDatabuf(buf, s, present, data_only=True)
            for i in range(k + m):
                sl = slice(i * s, (i + 1) * s)
                if i in missing and i >= k:
                    assert (buf[sl] == 0xA5).all()
                else:
                    assert np.array_equal(buf[sl], full[sl]), (missing, i)


def test_verify_databuf_oracle_parity_and_flips():
    k, m, s = 8, 3, 8192
    enc = RS.New(k, m)
    buf = _oracle_encode(k, m, _databuf(k, m, s, 3), s)
    assert enc.VerifyDatabuf(buf, s)
    for pos in (0, k * s - 1, k * s, (k + m) * s - 1, 5 * s + 77):
        bad = buf.copy()
        bad[pos] ^= 0x01
        assert not enc.VerifyDatabuf(bad, s), pos


def test_databuf_errors():
    enc = RS.New(4, 2)
    buf = np.zeros(6 * 64, np.uint8)
    with pytest.raises(RS.ErrShardNoData):
        enc.EncodeDatabuf(buf, 0)
    with pytest.raises(RS.ErrShardNoData):
        enc.ReconstructDatabuf(buf, 64, [0] * 6)
    with pytest.raises(RS.ErrTooFewShards):
        enc.ReconstructDatabuf(buf, 64, [1, 1, 1, 0, 0, 0])
    enc.ReconstructDatabuf(buf, 64, [1] * 6)  # nothing missing: no-op


def test_databuf_in_pinned_memory_zero_copy():
    """A databuf from hbec_host_alloc (the shim's pinned pool) is coded in
    place over PCIe; same bytes as the oracle."""
    k, m, s = 4, 2, 262144
    enc = RS.New(k, m)
    hb = RS.HostBuffer((k + m) * s)
    try:
        buf = hb.array
        buf[:] = _databuf(k, m, s, 91)
        want = _oracle_encode(k, m, buf.copy(), s)
        enc.EncodeDatabuf(buf, s)
        assert np.array_equal(buf, want)
        buf[:2 * s] = 0
        enc.ReconstructDatabuf(buf, s, [0, 0, 1, 1, 1, 1])
        assert np.array_equal(buf, want)
    finally:
        hb.free()


class _Rec:
    def __init__(self):
        self.calls = []

    def write(self, b):
        self.calls.append(bytes(b))

    def value(self):
        return b"".join(self.calls)


class _DiesAt:
    """Serves `data` until stripe `bad` (of `chunk` bytes per shard), then fails."""

    def __init__(self, data, chunk, bad):
        self.f = io.BytesIO(data)
        self.limit = chunk * bad

    def read(self, n):
        if self.f.tell() >= self.limit:
            raise IOError("peer gone")
        return self.f.read(min(n, self.limit - self.f.tell()))


def test_ec_reconstruct_stripe_with_no_shards_is_shard_no_data():
    """ecutils.go:103-113: when every body fails on a stripe, klauspost's
    Reconstruct returns ErrShardNoData (checkShards runs before the count);
    the stripes before it were written."""
    k, m, chunk = 4, 2, 1024
    length = 6 * k * chunk
    body = bytes(O.object_bytes(44, length))
    files = O.ec_split(k, m, body, chunk)
    bodies = [None] + [_DiesAt(f, chunk, 3) for f in files[1:]]
    dst = _Rec()
    with pytest.raises(RS.ErrShardNoData):
        E.ec_reconstruct(k, m, bodies, chunk, length, [dst], [0])
    assert dst.value() == files[0][:3 * chunk]
    with pytest.raises(O.ErrShardNoData):
        O.Encoder(k, m).reconstruct([np.zeros(0, np.uint8)] * (k + m))


def test_ec_glue_stripe_with_no_shards_is_shard_no_data():
    k, m, chunk = 4, 2, 1024
    length = 6 * k * chunk
    body = bytes(O.object_bytes(45, length))
    files = O.ec_split(k, m, body, chunk)
    bodies = [None] + [_DiesAt(f, chunk, 2) for f in files[1:]]
    out = _Rec()
    with pytest.raises(RS.ErrShardNoData):
        E.ec_glue(k, m, bodies, chunk, length, out)
    assert out.value() == body[:2 * k * chunk]


def test_pure_c_client_databuf_on_gpu(tmp_path):
    """tests/native/abi_smoke.c, the plain-C stand-in for the cgo shim, drives
    Encode / Reconstruct / ReconstructData / Verify through the databuf entry
    points on the GPU against the TESTING 3+2 and klauspost 5+5 known answers."""
    import subprocess
    from pathlib import Path

    from hummingbird_amd import _native as N

    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "abi_smoke"
    lib_dir = N.LIB_PATH.parent
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", str(root / "include"),
                    str(root / "tests" / "native" / "abi_smoke.c"), "-L", str(lib_dir), "-lhbec",
                    f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe), "gpu"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, (out.returncode, out.stderr)
    assert "databuf gpu ok" in out.stdout


@pytest.mark.parametrize("pinned", [False, True])
def test_percall_64_threads_coalesced_match_oracle(pinned):
    """64 threads each calling the plain per-call entries (EncodeDatabuf,
    Encode on consecutive slots, ReconstructDatabuf / ReconstructData) the way
    concurrent Stabilize / GET goroutines reach klauspost through the shim:
    calls on pinned databufs are coalesced into shared launches
    (hbec_coalesce_stats), pageable ones run per call, and every caller gets
    exactly its own bytes, checked against the oracle."""
    import ctypes as C
    import threading

    from hummingbird_amd import _native as N

    k, m, s = 4, 2, 65536
    n = 192
    enc = RS.New(k, m)
    stride = (k + m) * s
    hb = RS.HostBuffer(n * stride) if pinned else None
    pool = hb.array if pinned else np.zeros(n * stride, np.uint8)
    bufs = [pool[i * stride:(i + 1) * stride] for i in range(n)]
    for i, b in enumerate(bufs):
        b[:] = 0
        b[:k * s] = O.object_bytes(500 + i, k * s)
    want = [_oracle_encode(k, m, b.copy(), s) for b in bufs]
    g0, c0 = C.c_uint64(), C.c_uint64()
    N.lib().hbec_coalesce_stats(C.byref(g0), C.byref(c0))
    errors = []

    def work(t):
        try:
            for i in range(t, n, 64):
                b = bufs[i]
                if i % 2:
                    enc.EncodeDatabuf(b, s)
                else:
                    enc.Encode([b[j * s:(j + 1) * s] for j in range(k + m)])  # consecutive slots
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(64)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    for b, w in zip(bufs, want):
        assert np.array_equal(b, w)
    g1, c1 = C.c_uint64(), C.c_uint64()
    N.lib().hbec_coalesce_stats(C.byref(g1), C.byref(c1))
    if pinned:  # pinned databufs are grouped (one zero-copy launch per group)
        assert c1.value - c0.value == n
        assert g1.value - g0.value <= n
    else:  # pageable ones run per call: their staging copies parallel on the callers' threads
        assert c1.value - c0.value == 0
    # degraded reads / repair: two patterns interleaved, ReconstructData on some
    pats = [([0, 1, 1, 1, 1, 1], False), ([1, 1, 0, 1, 0, 1], False), ([0, 1, 1, 0, 1, 1], True)]
    for i, b in enumerate(bufs):
        present, _ = pats[i % 3]
        for j, p in enumerate(present):
            if not p:
                b[j * s:(j + 1) * s] = 0xEE

    def rec(t):
        try:
            for i in range(t, n, 64):
                present, data_only = pats[i % 3]
                enc.ReconstructDatabuf(bufs[i], s, present, data_only=data_only)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=rec, args=(t,)) for t in range(64)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    for i, (b, w) in enumerate(zip(bufs, want)):
        present, data_only = pats[i % 3]
        if data_only:
            assert np.array_equal(b[:k * s], w[:k * s]), i
            for j in range(k, k + m):
                if not present[j]:
                    assert (b[j * s:(j + 1) * s] == 0xEE).all()
        else:
            assert np.array_equal(b, w), i
    del bufs, pool
    if hb:
        hb.free()
