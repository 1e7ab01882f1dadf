"""Failure detection at the boundary (a GPU failure or OOM must
come back as an error code so the Go shim can fall back to klauspost's CPU
codec): allocation failures return HBEC_ERR_NOMEM, nothing is half-written,
and the very next call on the same thread succeeds (a failed HIP call must not
leave its code in the runtime's last-error slot for the next launch check)."""
import ctypes as C

import numpy as np
import pytest
import torch

from hummingbird_amd import _native as N
from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    yield
    torch.cuda.empty_cache()


def _encode_ok(enc, k, m, s=4096, seed=0):
    rng = np.random.default_rng(seed)
    sh = [rng.integers(0, 256, s, dtype=np.uint8) for _ in range(k)] + [np.zeros(s, np.uint8) for _ in range(m)]
    enc.Encode(sh)
    want = CO.apply(CO.build_matrix(k, m)[k:], sh[:k])
    assert all(np.array_equal(sh[k + r], want[r]) for r in range(m))


def test_pinned_host_alloc_failure_is_nomem_and_recovers():
    p = C.c_void_p()
    # 1 PiB: beyond the 47-bit user address space, so it fails before pinning anything
    rc = N.lib().hbec_host_alloc(1 << 50, C.byref(p))
    assert rc in (N.ERR_NOMEM, N.ERR_DEVICE), rc
    assert p.value is None
    assert "hipHostMalloc" in N.last_error()
    assert N.lib().hbec_host_alloc(1 << 20, C.byref(p)) == N.HBEC_OK
    N.lib().hbec_host_free(p)
    _encode_ok(RS.New(4, 2), 4, 2, seed=1)


def test_device_oom_is_nomem_and_next_call_succeeds():
    """A stripe plan's tile records live in HBM (hbec_plan_stripes, one 32-B
    record per tile).  With HBM nearly full, a plan whose records need 1 GiB
    fails with ErrNoMem and allocates nothing, while an unaligned 4+2 Verify
    (gf_odd, no scratch) and a k = 17 Verify (gf_verify_wide, no scratch since
    round 3) still succeed.  With the memory back, the same plan is made, and
    an aligned pipelined encode succeeds (the launch check sees no stale
    error from the failed allocation)."""
    k, m, n, s = 17, 2, 64, (1 << 16) + 1  # k > 16, odd shard length: gf_verify_wide
    enc = RS.New(k, m)
    e42, s42 = RS.New(4, 2), 1001
    small = torch.empty((8, 6 * s42 + 3), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(small, 6 * s42 + 3)
    v42 = [(small.data_ptr() + 3 + i * s42, small.stride(0)) for i in range(6)]
    B.encode_views(e42, v42, 8, s42)
    f42 = torch.zeros(8, dtype=torch.int32, device="cuda")
    objs = torch.empty((n, k * s + 1), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * s + 1)
    parity = torch.empty((n, m * s + 1), dtype=torch.uint8, device="cuda")
    views = [(objs.data_ptr() + 1 + j * s, objs.stride(0)) for j in range(k)]
    views += [(parity.data_ptr() + 1 + r * s, parity.stride(0)) for r in range(m)]
    B.encode_views(enc, views, n, s)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    # 512 aligned 4+2 stripes of 64 MiB shards: 32 Mi tile records = 1 GiB in
    # HBM (the plan only records addresses; it is never run)
    big = [(small.data_ptr() - (small.data_ptr() % 256), 64 << 20)] * 512

    free, _ = torch.cuda.mem_get_info()
    hog = None
    for slack in (256 << 20, 512 << 20, 768 << 20):  # leave less than the plan's 1 GiB
        try:
            hog = torch.empty(free - slack, dtype=torch.uint8, device="cuda")
            break
        except RuntimeError:
            continue
    assert hog is not None, "could not fill HBM for the test"
    try:
        with pytest.raises(RS.ErrNoMem):
            B.StripePlan(e42, big)
        assert "hipMalloc plan tiles" in N.last_error()
        B.verify_views(e42, v42, 8, s42, f42)
        B.verify_views(enc, views, n, s, flags)
        torch.cuda.synchronize()
        assert int(f42.count_nonzero()) == 0 and int(flags.count_nonzero()) == 0
    finally:
        del hog
        torch.cuda.empty_cache()

    plan = B.StripePlan(e42, big)  # the same call, memory back
    del plan
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0
    a = torch.empty((64, 4 << 18), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(a, 4 << 18)
    p = torch.empty((64, 2 << 18), dtype=torch.uint8, device="cuda")
    B.encode_objects(e42, a, p, 1 << 18)  # aligned 4+2: the pipelined kernel launch check
    torch.cuda.synchronize()
    want, _ = CO.encode_batch(4, 2, a[:2].cpu().numpy())
    assert np.array_equal(p[:2].cpu().numpy(), want)
