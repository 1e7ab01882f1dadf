"""N>1 control path of bench.py on CPU (gloo, world_size 2).

The hot path is partitioned, not exchanged: each rank owns a contiguous range
of global objects and the only collectives are the barrier and the
max-over-ranks timing reduction.  These tests run that logic with gloo."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_per_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, r, local = bench.dist_env()
        first, n = bench.partition(n_per_rank, r)
        dist.barrier()
        elapsed = 1.0 + r  # rank 1 is slower
        vals = bench.max_over_ranks(dist, [elapsed, 0.5 * (r + 1), 0.0 if r == 0 else 1.0], "cpu")
        q.put((r, w, local, first, n, vals))
    finally:
        dist.destroy_process_group()


def test_partition_and_max_over_ranks_gloo():
    world, n_per_rank = 2, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    ranges = [(first, first + n) for _, _, _, first, n, _ in res]
    assert ranges == [(0, 4096), (4096, 8192)]  # disjoint, contiguous, covering
    for r, w, local, _, _, vals in res:
        assert w == world and local == r
        assert vals == [2.0, 1.0, 1.0]  # every rank sees the max


def test_single_process_helpers():
    assert bench.partition(4096, 0) == (0, 4096)
    assert bench.partition(4096, 7) == (7 * 4096, 4096)
    assert bench.max_over_ranks(None, [1.0, 2.0], "cpu") == [1.0, 2.0]
