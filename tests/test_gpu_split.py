"""bench.batch_split (BASELINE configs[4]) on the GPU with a world-size-1 gloo
group: allocation agreement, the split's copy path, the partition encode on
libhbec's kernel and rank 0's whole-batch parity check.  The RCCL P2P rounds
themselves are covered on CPU by tests/test_dist.py (gloo, world 2 and 3)."""
import os
import socket

import pytest
import torch

import bench

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_batch_split_single_rank_gpu():
    import torch.distributed as dist

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        res = bench.batch_split(dist, 4, 2, 1 << 20, 64, 1, 0, "cpu")
    finally:
        dist.destroy_process_group()
    assert "skipped" not in res, res
    assert res["parity_ok"] is True
    assert res["objects"] == 64 and res["objects_per_rank_max"] == 64
    assert res["encode_ms"] > 0


def test_config5_full_partition_one_gpu_full_oracle():
    """BASELINE configs[4] at G=1: all 65 536 x 1 MiB 4+2 objects (64 GiB data
    + 32 GiB parity) resident on one GPU and encoded by libhbec in ONE batch
    call.  EVERY object's parity is compared byte for byte with the CPU
    oracle's encode of the same bytes (oracle/gf_oracle.c, 1024-object chunks
    streamed to the host), every object passes the GPU Verify kernel, and a
    sample of objects is checked to be the oracle's own splitmix inputs."""
    import numpy as np

    import fullcheck
    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS
    from oracle import coracle as CO

    torch.cuda.set_device(0)
    torch.cuda.empty_cache()
    k, m, size, n = 4, 2, 1 << 20, 65536
    s = size // k
    enc = RS.New(k, m)
    objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
    parity = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    try:
        B.fill_splitmix(objs, size)
        B.encode_objects(enc, objs, parity, s)
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.verify_views(enc, B.shard_views(objs, k, s) + B.shard_views(parity, m, s), n, s, flags)
        torch.cuda.synchronize()
        assert int(flags.count_nonzero().item()) == 0
        rng = np.random.default_rng(0x48424543)
        picks = sorted({0, 1, n // 2, n - 2, n - 1, *rng.integers(0, n, 27).tolist()})
        host = objs.index_select(0, torch.tensor(picks, device="cuda")).cpu().numpy()
        for i, o in enumerate(picks):  # the GPU's inputs are the oracle's splitmix objects
            assert np.array_equal(host[i], CO.fill_objects(o, 1, size)[0]), o
        assert fullcheck.encode_parity_matches(k, m, objs, parity) == n
    finally:
        del objs, parity
        torch.cuda.empty_cache()


def test_config5_leg_single_rank():
    """bench.config5 (the JSON line's `config5` object) on one GPU with a
    small partition: timing fields and the GPU-side parity check."""
    torch.cuda.set_device(0)
    res = bench.config5(None, 4, 2, 1 << 20, 512, 1, 0, "cuda", reps=2)
    assert "skipped" not in res, res
    assert res["parity_ok"] is True and res["objects"] == 512 and res["objects_per_gpu_max"] == 512
    assert res["value_GiB_s"] > 0 and 0 < res["per_gpu_roofline"]["frac"] < 1.0
