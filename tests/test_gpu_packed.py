"""gf_apply_packed (short shards: wave tiles across objects) against the CPU
oracle: shard lengths from one element (16 B) up to the kernel's limit, odd
element counts (S/16 not a power of two, so objects straddle lanes at every
offset), one object, partial last tiles, padded object strides, and
reconstruct with survivors in two arrays and outputs in a third."""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    yield


SHAPES = [(1, 1), (2, 1), (3, 2), (4, 2), (5, 3), (8, 3), (6, 2)]
# 5 <= K <= 8 up to 32 KiB since round 6: both sides of the old 3 KiB limit,
# of the pipelined kernel's 3 KiB tiles and of the new 32 KiB limit
LENS = [16, 48, 96, 256, 512, 1008, 1024, 1040, 2032, 3056, 3072, 4096, 4112, 6160, 8192, 12304, 16384, 32768, 32784]


def _packed(k, s):
    """The dispatch rule of kernels.hip is_packed_shape (no device needed at
    collection): S < 2 KiB for K <= 4, S <= 32 KiB for 5 <= K <= 8
    (tuning.h HBEC_PACKED_MAX_BIG)."""
    return s % 16 == 0 and s < (2048 if k <= 4 else 32784)


def _cases():
    for k, m in SHAPES:
        for s in LENS:
            if _packed(k, s):
                yield k, m, s


@pytest.mark.parametrize("k,m,s", list(_cases()))
@pytest.mark.parametrize("n", [1, 7, 333])
def test_packed_encode_matches_oracle(k, m, s, n):
    if s > 4096 and n == 333:
        n = 37  # the oracle's time, not coverage: 37 objects still span many tiles
    pad = 48  # object rows longer than k*S: the views' strides differ from S
    objs = torch.empty((n, k * s + pad), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s + pad, first=k * 1000 + s)
    parity = torch.full((n, m * s + pad), 0xC5, dtype=torch.uint8, device="cuda")
    enc = RS.New(k, m)
    views = [(objs.data_ptr() + j * s, objs.stride(0)) for j in range(k)]
    views += [(parity.data_ptr() + r * s, parity.stride(0)) for r in range(m)]
    assert B.kernel_info(k, m, s)["kind"] == "packed"
    B.encode_views(enc, views, n, s)
    torch.cuda.synchronize()
    host = objs.cpu().numpy()
    want, _ = CO.encode_batch(k, m, np.ascontiguousarray(host[:, :k * s]))
    got = parity.cpu().numpy()
    assert np.array_equal(got[:, :m * s], want)
    assert (got[:, m * s:] == 0xC5).all()  # nothing written past the last shard


@pytest.mark.parametrize("k,m,s", [(8, 3, 512), (4, 2, 1024), (4, 2, 48), (3, 2, 2032), (8, 3, 3056), (8, 3, 4096),
                                   (6, 3, 12304), (8, 3, 32768)])
def test_packed_reconstruct_three_arrays(k, m, s):
    n = 501
    enc = RS.New(k, m)
    objs = torch.empty((n, k * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s, first=s)
    parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    B.encode_objects(enc, objs, parity, s)
    missing = [0, k - 1, k][:m]
    rebuilt = torch.zeros((n, len(missing) * s), dtype=torch.uint8, device="cuda")
    views = B.shard_views(objs, k, s) + B.shard_views(parity, m, s)
    for slot, i in enumerate(missing):
        views[i] = (rebuilt.data_ptr() + slot * s, rebuilt.stride(0))
    B.reconstruct_views(enc, views, [0 if i in missing else 1 for i in range(k + m)], n, s)
    torch.cuda.synchronize()
    for slot, i in enumerate(missing):
        src = objs[:, i * s:(i + 1) * s] if i < k else parity[:, (i - k) * s:(i - k + 1) * s]
        assert torch.equal(rebuilt[:, slot * s:(slot + 1) * s], src), i


def test_packed_kernel_is_selected_for_short_shards():
    assert B.kernel_info(8, 3, 512)["kind"] == "packed"
    assert B.kernel_info(4, 2, 1024)["kind"] == "packed"
    assert B.kernel_info(4, 2, 2048)["kind"] == "pipelined"
    assert B.kernel_info(8, 3, 3072)["kind"] == "packed"
    assert B.kernel_info(8, 3, 32768)["kind"] == "packed"
    assert B.kernel_info(8, 3, 32784)["kind"] == "pipelined"
    assert B.kernel_info(8, 4, 4096)["kind"] != "packed"  # no 4-row packed instance


def _verify_packed(k, s):
    """verify.hip is_verify_packed_shape: S < max(verify tile, 2 KiB), i.e.
    S < 4 KiB for K <= 4 and S < 2 KiB for 5 <= K <= 8."""
    return s % 16 == 0 and s < (4096 if k <= 4 else 2048)


def _verify_cases():
    for k, m in SHAPES + [(4, 4), (8, 4), (2, 4)]:
        for s in LENS + [3072, 4080]:
            if _verify_packed(k, s):
                yield k, m, s


@pytest.mark.parametrize("k,m,s", list(_verify_cases()))
@pytest.mark.parametrize("n", [1, 7, 333])
def test_packed_verify_oracle_parity_and_flips(k, m, s, n):
    """gf_verify_packed on parity the oracle computed (not the GPU encoder):
    every object clean, then single-byte flips in chosen objects' data or
    parity shards flag exactly those objects — objects share a wave here, so
    each lane must flag its own object."""
    pad = 32
    rng = np.random.default_rng(k * 7919 + m * 131 + s + n)
    data = rng.integers(0, 256, size=(n, k * s + pad), dtype=np.uint8)
    want, _ = CO.encode_batch(k, m, np.ascontiguousarray(data[:, :k * s]))
    par = np.zeros((n, m * s + pad), dtype=np.uint8)
    par[:, :m * s] = want
    objs = torch.from_numpy(data).cuda()
    parity = torch.from_numpy(par).cuda()
    enc = RS.New(k, m)
    views = [(objs.data_ptr() + j * s, objs.stride(0)) for j in range(k)]
    views += [(parity.data_ptr() + r * s, parity.stride(0)) for r in range(m)]
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0
    bad = sorted(set(rng.integers(0, n, size=min(n, 5)).tolist()))
    for o in bad:
        shard = int(rng.integers(0, k + m))
        off = int(rng.integers(0, s))
        if shard < k:
            objs[o, shard * s + off] ^= 0x5A
        else:
            parity[o, (shard - k) * s + off] ^= 0x5A
    # bytes outside the shards (row padding) are not part of any object
    objs[:, k * s:] ^= 0xFF
    parity[:, m * s:] ^= 0xFF
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert torch.nonzero(flags).flatten().tolist() == bad
