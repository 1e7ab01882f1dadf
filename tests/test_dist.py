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


def _split_worker(rank, world, port, n_global, row, chunk, q):
    """scatter_objects / gather_rows (hummingbird_amd/split.py) over gloo with
    CPU tensors: the same P2P rounds bench.py runs over RCCL for configs[4]."""
    from hummingbird_amd import split as SP

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, n = SP.object_range(n_global, world, rank)
        batch = None
        if rank == 0:
            batch = torch.arange(n_global * row, dtype=torch.int64).remainder(251).to(torch.uint8).view(n_global, row)
        part = torch.zeros((n, row), dtype=torch.uint8)
        SP.scatter_objects(dist, batch, part, n_global, chunk_bytes=chunk)
        want = torch.arange(first * row, (first + n) * row, dtype=torch.int64).remainder(251).to(torch.uint8)
        got_ok = bool(torch.equal(part.view(-1), want))
        # "parity": a per-object function of the received rows, gathered back
        res = (part[:, :3].to(torch.int32) * 7 + rank).to(torch.uint8).contiguous()
        dest = torch.zeros((n_global, 3), dtype=torch.uint8) if rank == 0 else None
        SP.gather_rows(dist, res, dest, n_global, chunk_bytes=chunk)
        gather_ok = True
        if rank == 0:
            for r in range(world):
                f, c = SP.object_range(n_global, world, r)
                src_rows = batch[f:f + c, :3].to(torch.int32)
                gather_ok &= bool(torch.equal(dest[f:f + c], (src_rows * 7 + r).to(torch.uint8)))
        q.put((rank, first, n, got_ok, gather_ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_global,chunk", [(2, 8, 64), (3, 10, 48), (3, 2, 1 << 20)])
def test_batch_split_scatter_gather_gloo(world, n_global, chunk):
    row = 16  # chunk // row objects per P2P message: several rounds per peer
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, n_global, row, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert sum(n for _, _, n, _, _ in res) == n_global
    assert all(ok and gok for *_, ok, gok in res)


def test_object_range_partition():
    from hummingbird_amd import split as SP

    for n_global in (0, 1, 7, 65536, 65537):
        for world in (1, 2, 3, 8):
            parts = [SP.object_range(n_global, world, r) for r in range(world)]
            assert parts[0][0] == 0
            for (f0, n0), (f1, _) in zip(parts, parts[1:]):
                assert f0 + n0 == f1
            assert sum(n for _, n in parts) == n_global
            assert max(n for _, n in parts) - min(n for _, n in parts) <= 1
    assert SP.object_range(65536, 8, 7) == (7 * 8192, 8192)
    with pytest.raises(ValueError):
        SP.object_range(4, 0, 0)


def _clean_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _bench_cmd(*args):
    import subprocess
    import sys
    from pathlib import Path

    root = Path(bench.__file__).resolve().parent
    return subprocess.run([sys.executable, str(root / "bench.py"), *args], env=_clean_env(), cwd=str(root),
                          capture_output=True, text=True, timeout=300)


def test_bench_gpus_without_launcher_spawns_ranks():
    """`python bench.py --gpus 2` with no launcher env starts 2 ranks itself
    (torch.distributed.run in a child process) and reports n_gpus 2."""
    import json

    r = _bench_cmd("--gpus", "2", "--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2
    assert lines[0]["per_rank"] == [[0.0, 0.0], [1.0, 10.0]]  # every rank's launch times, in rank order


def test_bench_single_gpu_dry_run():
    import json

    r = _bench_cmd("--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["n_gpus"] == 1 and line["ranks_seen"] == 1


def test_bench_refuses_launcher_world_mismatch():
    import subprocess
    import sys
    from pathlib import Path

    root = Path(bench.__file__).resolve().parent
    env = _clean_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       cwd=str(root), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
