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
