"""Batch split across the GPUs of one node (BASELINE configs[4]).

Objects are independent (objectserver/ecutils.go:38-70: every stripe is
encoded on its own), so a batch that lands on one GPU is *partitioned*, never
reduced: rank r owns the contiguous global objects [first_r, first_r + n_r).
The only data movement is the split itself, point-to-point over xGMI:

  scatter_objects  — the holder (rank `src`) sends each peer its slice of
                     object rows; on ROCm the "nccl" backend is RCCL, so each
                     peer's slice travels over its own xGMI link, all links
                     at once.
  gather_rows      — the reverse for results (parity / rebuilt shards).

Messages are cut into chunks of whole objects (`chunk_bytes`, default
256 MiB).  Chunk c of every peer forms one P2P group, so a group holds at most
world-1 operations, no RCCL call carries more than one chunk, and all links
stream at once.  No collective ever touches the GF arithmetic: each rank then
runs libhbec's kernels on its own partition.  The holder's own slice is not
sent anywhere (it is a view / device copy).

The functions take any torch.distributed process-group-like module (the
`torch.distributed` module itself, as bench.py passes it), so the same code is
tested on CPU with gloo (tests/test_dist.py) and runs on RCCL on the GPU node.
"""
from __future__ import annotations


def object_range(n_global: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous partition of n_global objects over `world` ranks: the first
    n_global % world ranks take one extra object.  Returns (first, count)."""
    if world <= 0 or not 0 <= rank < world or n_global < 0:
        raise ValueError("bad partition arguments")
    base, extra = divmod(n_global, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def _chunks(n_rows: int, row_bytes: int, chunk_bytes: int):
    per = max(1, chunk_bytes // max(1, row_bytes))
    for a in range(0, n_rows, per):
        yield a, min(n_rows, a + per)


def _p2p(dist, ops):
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def scatter_objects(dist, batch, out, n_global: int, src: int = 0, chunk_bytes: int = 256 << 20) -> None:
    """Rank `src` holds `batch` [n_global, L] (rows = objects); every rank
    receives its object_range rows into `out` [n_r, L].  `batch` is ignored on
    other ranks (pass None)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    first, n = object_range(n_global, world, rank)
    if out.dim() != 2 or out.shape[0] != n or not out.is_contiguous():
        raise ValueError(f"rank {rank}: out must be a contiguous [{n}, L] tensor")
    row = out.shape[1] * out.element_size()
    if rank == src:
        if batch is None or batch.dim() != 2 or batch.shape[0] != n_global or batch.shape[1] != out.shape[1]:
            raise ValueError("src rank: batch must be [n_global, L] with the same row length as out")
        out.copy_(batch[first:first + n])
        plans = {p: list(_chunks(object_range(n_global, world, p)[1], row, chunk_bytes))
                 for p in range(world) if p != src}
        for c in range(max((len(v) for v in plans.values()), default=0)):
            ops = []
            for peer, ch in plans.items():
                if c < len(ch):
                    pf = object_range(n_global, world, peer)[0]
                    a, b = ch[c]
                    ops.append(dist.P2POp(dist.isend, batch[pf + a:pf + b], peer))
            _p2p(dist, ops)
    else:
        for a, b in _chunks(n, row, chunk_bytes):
            _p2p(dist, [dist.P2POp(dist.irecv, out[a:b], src)])


def gather_rows(dist, part, dest, n_global: int, dst: int = 0, chunk_bytes: int = 256 << 20) -> None:
    """Inverse of scatter_objects: every rank's `part` [n_r, W] lands in rows
    object_range(rank) of `dest` [n_global, W] on rank `dst` (None elsewhere)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    first, n = object_range(n_global, world, rank)
    if part.dim() != 2 or part.shape[0] != n or not part.is_contiguous():
        raise ValueError(f"rank {rank}: part must be a contiguous [{n}, W] tensor")
    row = part.shape[1] * part.element_size()
    if rank == dst:
        if dest is None or dest.dim() != 2 or dest.shape[0] != n_global or dest.shape[1] != part.shape[1]:
            raise ValueError("dst rank: dest must be [n_global, W] with the same row length as part")
        dest[first:first + n].copy_(part)
        plans = {p: list(_chunks(object_range(n_global, world, p)[1], row, chunk_bytes))
                 for p in range(world) if p != dst}
        for c in range(max((len(v) for v in plans.values()), default=0)):
            ops = []
            for peer, ch in plans.items():
                if c < len(ch):
                    pf = object_range(n_global, world, peer)[0]
                    a, b = ch[c]
                    ops.append(dist.P2POp(dist.irecv, dest[pf + a:pf + b], peer))
            _p2p(dist, ops)
    else:
        for a, b in _chunks(n, row, chunk_bytes):
            _p2p(dist, [dist.P2POp(dist.isend, part[a:b], dst)])
