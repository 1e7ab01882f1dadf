"""The pipelined stripe loops (csrc/ecutils.cpp): stripe i+1 is read while
stripe i is on the GPU, so these check what a caller of ecutils.go can
observe across many stripes — output bytes, the sequence of writes, and the
error paths — against the oracle's restatement of ecutils.go:26-186.
"""
import io

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


class Rec:
    """Writer recording each write call separately."""

    def __init__(self):
        self.calls = []

    def write(self, b):
        self.calls.append(bytes(b))

    def value(self):
        return b"".join(self.calls)


class FailingReader:
    """Reads from a bytes body; raises once `fail_at` bytes have been served."""

    def __init__(self, data, fail_at=None):
        self.f = io.BytesIO(data)
        self.fail_at = fail_at
        self.served = 0

    def read(self, n):
        if self.fail_at is not None and self.served >= self.fail_at:
            raise IOError("body broke")
        if self.fail_at is not None:
            n = min(n, self.fail_at - self.served)
        b = self.f.read(n)
        self.served += len(b)
        return b


@pytest.mark.parametrize("k,m,chunk,length", [(4, 2, 1024, 40_000), (8, 3, 4096, 300_001), (3, 2, 1000, 7),
                                              (4, 2, 65536, 4 * 65536 * 5), (10, 4, 1003, 51_234)])
def test_split_many_stripes_write_sequence(k, m, chunk, length):
    body = bytes(O.object_bytes(k * 31 + m, length))
    ws = [Rec() for _ in range(k + m)]
    E.ec_split(k, m, io.BytesIO(body), chunk, length, ws)
    files = O.ec_split(k, m, body, chunk)
    stripes = -(-length // (k * chunk))
    for i in range(k + m):
        assert ws[i].value() == files[i]
        assert len(ws[i].calls) == stripes  # one write per stripe, in stripe order


@pytest.mark.parametrize("cut_stripe", [0, 1, 4])
def test_split_short_read_writes_complete_stripes_first(cut_stripe):
    k, m, chunk = 4, 2, 1024
    stripe = k * chunk
    length = 8 * stripe
    body = bytes(O.object_bytes(5, length))
    avail = cut_stripe * stripe + 100  # the read of stripe `cut_stripe` comes up short
    ws = [Rec() for _ in range(k + m)]
    with pytest.raises(RS.ErrUnexpectedEOF):
        E.ec_split(k, m, io.BytesIO(body[:avail]), chunk, length, ws)
    want = O.ec_split(k, m, body[:cut_stripe * stripe], chunk) if cut_stripe else [b""] * (k + m)
    for i in range(k + m):
        assert ws[i].value() == want[i]


def test_split_reader_error_mid_object():
    k, m, chunk = 4, 2, 2048
    length = 6 * k * chunk
    body = bytes(O.object_bytes(9, length))
    ws = [Rec() for _ in range(k + m)]
    with pytest.raises(RS.ErrIO):
        E.ec_split(k, m, FailingReader(body, fail_at=3 * k * chunk), chunk, length, ws)
    want = O.ec_split(k, m, body[:3 * k * chunk], chunk)
    assert [w.value() for w in ws] == want


def test_split_failing_writer_dropped_midway():
    k, m, chunk = 4, 2, 1024
    length = 10 * k * chunk
    body = bytes(O.object_bytes(11, length))

    class Breaks(Rec):
        def write(self, b):
            if len(self.calls) == 3:
                raise IOError("peer went away")
            super().write(b)

    ws = [Rec() for _ in range(k + m)]
    ws[1] = Breaks()
    ws[5] = Breaks()
    E.ec_split(k, m, io.BytesIO(body), chunk, length, ws)
    files = O.ec_split(k, m, body, chunk)
    for i in range(k + m):
        if i in (1, 5):
            assert ws[i].value() == files[i][:3 * chunk]
        else:
            assert ws[i].value() == files[i]


@pytest.mark.parametrize("k,m,chunk,length,erased", [(4, 2, 1024, 50_000, (0, 5)), (8, 3, 4096, 400_000, (1, 2, 9)),
                                                     (4, 2, 1000, 9_999, (3,)), (3, 2, 100, 7, (0, 1)),
                                                     (10, 4, 1003, 51_234, (0, 9, 11, 13)),
                                                     (17, 3, 2048, 200_000, (0, 16, 19))])
def test_reconstruct_many_stripes(k, m, chunk, length, erased):
    body = bytes(O.object_bytes(k + 100 * m, length))
    files = O.ec_split(k, m, body, chunk)
    bodies = [None if i in erased else io.BytesIO(files[i]) for i in range(k + m)]
    dsts = [Rec() for _ in erased]
    E.ec_reconstruct(k, m, bodies, chunk, length, dsts, list(erased))
    for d, i in zip(dsts, erased):
        assert d.value() == files[i]


def test_reconstruct_body_failure_is_per_stripe():
    """ecutils.go:103-109: a body whose read fails is missing for that stripe
    only (never marked failed) and is read again on the next stripe."""
    k, m, chunk = 4, 2, 1024
    length = 6 * k * chunk
    body = bytes(O.object_bytes(21, length))
    files = O.ec_split(k, m, body, chunk)

    class FlakyOnce:
        def __init__(self, data, bad_stripe):
            self.f = io.BytesIO(data)
            self.bad = bad_stripe
            self.calls = 0

        def read(self, n):
            stripe = self.f.tell() // chunk
            if stripe == self.bad and self.calls == 0:
                self.calls += 1
                self.f.seek(chunk, 1)  # the stripe's bytes are consumed by the failed read
                raise IOError("flaky")
            return self.f.read(n)

    bodies = [io.BytesIO(f) for f in files]
    bodies[2] = FlakyOnce(files[2], bad_stripe=3)
    bodies[0] = None  # erased: rebuilt every stripe
    dsts = [Rec()]
    E.ec_reconstruct(k, m, bodies, chunk, length, dsts, [0])
    assert dsts[0].value() == files[0]


@pytest.mark.parametrize("k,m,chunk,length,lost", [(4, 2, 1024, 70_000, ()), (4, 2, 1024, 70_000, (1, 4)),
                                                   (8, 3, 4096, 333_333, (0, 7, 8)), (3, 2, 10, 7, (2,)),
                                                   (10, 4, 1003, 51_234, (2, 5, 10, 12)),
                                                   (17, 3, 2048, 200_000, (0, 8, 16))])
def test_glue_many_stripes(k, m, chunk, length, lost):
    body = bytes(O.object_bytes(k * 7 + len(lost), length))
    files = O.ec_split(k, m, body, chunk)
    bodies = [None if i in lost else io.BytesIO(files[i]) for i in range(k + m)]
    out = Rec()
    E.ec_glue(k, m, bodies, chunk, length, out)
    assert out.value() == body


def test_glue_body_failing_midway_stays_failed():
    k, m, chunk = 4, 2, 1024
    length = 8 * k * chunk
    body = bytes(O.object_bytes(33, length))
    files = O.ec_split(k, m, body, chunk)
    bodies = [io.BytesIO(f) for f in files]
    bodies[1] = FailingReader(files[1], fail_at=3 * chunk)
    out = Rec()
    E.ec_glue(k, m, bodies, chunk, length, out)
    assert out.value() == body


def _loop_cases():
    rng = np.random.default_rng(1610)
    for _ in range(20):
        k = int(rng.integers(1, 13))
        m = int(rng.integers(1, 5))
        chunk = int(rng.choice([1, 7, 100, 1000, 1024, 4096, 65536]))
        length = int(rng.integers(1, 200_000))
        lost = sorted(rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False).tolist())
        yield k, m, chunk, length, lost


@pytest.mark.parametrize("k,m,chunk,length,lost", list(_loop_cases()))
def test_stripe_loops_random_against_oracle(k, m, chunk, length, lost):
    """Random shapes through all three C++ stripe loops on the GPU codec:
    ecSplit's shard files equal the oracle's, ecGlue restores the object with
    `lost` shard files missing, ecReconstruct rebuilds exactly those files."""
    body = bytes(O.object_bytes(k * 997 + m * 13 + chunk, length))
    ws = [Rec() for _ in range(k + m)]
    E.ec_split(k, m, io.BytesIO(body), chunk, length, ws)
    files = O.ec_split(k, m, body, chunk)
    assert [w.value() for w in ws] == [bytes(f) for f in files]
    out = Rec()
    E.ec_glue(k, m, [None if i in lost else io.BytesIO(files[i]) for i in range(k + m)], chunk, length, out)
    assert out.value() == body
    dsts = [Rec() for _ in lost]
    E.ec_reconstruct(k, m, [None if i in lost else io.BytesIO(files[i]) for i in range(k + m)], chunk, length,
                     dsts, list(lost))
    assert [d.value() for d in dsts] == [bytes(files[i]) for i in lost]


def _range_bodies(files, k, chunk, start, end):
    shard_start, _ = O.range_chunk_align(start, end, chunk, k)
    return [None if f is None else io.BytesIO(f[shard_start:]) for f in files]


@pytest.mark.parametrize("k,m,chunk,length", [(4, 2, 1024, 40_000), (8, 3, 4096, 300_001), (2, 1, 10, 80),
                                              (10, 4, 1003, 51_234)])
def test_glue_range_is_the_slice(k, m, chunk, length):
    """CopyRange decode (hbec_ec_glue_range) returns object[start:end] from
    ranged shard bodies, healthy and with m shards lost (GPU ReconstructData),
    and agrees with the oracle's restatement."""
    body = bytes(O.object_bytes(k * 13 + m, length))
    files = O.ec_split(k, m, body, chunk)
    rng = np.random.default_rng(length)
    stripe = k * chunk
    ranges = [(0, length), (0, 1), (length - 1, length), (stripe, 2 * stripe), (stripe - 1, stripe + 1), (3, 3)]
    ranges += [tuple(int(x) for x in sorted(rng.integers(0, length + 1, 2))) for _ in range(12)]
    for start, end in ranges:
        for lose in (False, True):
            fs = list(files)
            if lose:
                for i in rng.choice(k + m, m, replace=False):
                    fs[i] = None
            out = Rec()
            E.ec_glue_range(k, m, _range_bodies(fs, k, chunk, start, end), chunk, length, start, end, out)
            assert out.value() == body[start:end]
            assert out.value() == O.ec_glue_range(k, m, fs, chunk, length, start, end)


@pytest.mark.parametrize("k,m,chunk,length", [(4, 2, 1024, 40_000), (8, 3, 4096, 300_001), (2, 1, 10, 80),
                                              (10, 4, 1003, 51_234), (1, 1, 7, 50)])
def test_copy_range_is_the_reference_bytes(k, m, chunk, length):
    """hbec_ec_copy_range (the byte-exact CopyRange drop-in) returns what
    ecObject.CopyRange writes (oracle.ec_copy_range, ecobj.go:207-267, the
    shard/object unit mix included) for healthy and degraded shard sets, from
    the ranged shard bodies "bytes=shardStart-shardEnd"; and it equals
    object[start:end] exactly on the ranges the reference's arithmetic maps to
    the object slice (oracle.copy_range_is_object_slice), where
    hbec_ec_glue_range gives the same bytes."""
    body = bytes(O.object_bytes(k * 17 + m, length))
    files = O.ec_split(k, m, body, chunk)
    rng = np.random.default_rng(length + k)
    stripe = k * chunk
    ranges = [(0, length), (0, 1), (0, chunk), (1, chunk // 2 + 1), (stripe, 2 * stripe), (stripe + 3, stripe + 9),
              (length - 1, length), (3, 3)]
    ranges += [tuple(int(x) for x in sorted(rng.integers(0, length + 1, 2))) for _ in range(16)]
    n_agree = 0
    for start, end in ranges:
        for lose in (False, True):
            fs = list(files)
            if lose:
                for i in rng.choice(k + m, m, replace=False):
                    fs[i] = None
            shard_start, shard_end = O.range_chunk_align(start, end, chunk, k)
            shard_end = min(shard_end, length)
            bodies = [None if b is None else io.BytesIO(b)
                      for b in (O.http_range_body(f, shard_start, shard_end) for f in fs)]
            out = Rec()
            E.ec_copy_range(k, m, bodies, chunk, length, start, end, out)
            want = O.ec_copy_range(k, m, fs, chunk, length, start, end)
            assert out.value() == want, (start, end, lose)
            if O.copy_range_is_object_slice(k, chunk, length, start, end):
                assert want == body[start:end]
                n_agree += not lose
    assert n_agree > 0


def test_glue_range_reference_writer_kats(kats):
    """TestRangeBytesWriter's vectors (ecobj_test.go:332-358) through the
    library: a 1+1 object "THIS IS A TEST" glued with chunk sizes 1..19 (the
    writer sees pieces of that size, as io.CopyBuffer's buffer)."""
    rb = kats["range_bytes_writer"]
    data = rb["data"].encode()
    for chunk in rb["buffer_sizes"]:
        files = O.ec_split(1, 1, data, chunk)
        for off, length, want in rb["cases"]:
            out = Rec()
            E.ec_glue_range(1, 1, _range_bodies(files, 1, chunk, off, off + length), chunk, len(data), off,
                            off + length, out)
            assert out.value() == want.encode()
            if chunk > 1:
                assert all(len(c) <= chunk for c in out.calls)


def test_glue_range_arguments_and_writers():
    k, m, chunk, length = 4, 2, 100, 2_000
    body = bytes(O.object_bytes(3, length))
    files = O.ec_split(k, m, body, chunk)
    for start, end in ((5, 4), (-1, 3), (0, length + 1)):
        with pytest.raises(RS.ErrInvalidArg):
            E.ec_glue_range(k, m, _range_bodies(files, k, chunk, 0, 1), chunk, length, start, end, Rec())

    class Broken:
        def write(self, b):
            raise IOError("client went away")

    good = Rec()
    E.ec_glue_range(k, m, _range_bodies(files, k, chunk, 450, 1750), chunk, length, 450, 1750, Broken(), None,
                    good)
    assert good.value() == body[450:1750]  # a failing or nil writer does not stop the others
