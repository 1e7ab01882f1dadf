"""BASELINE configs[3] at full size, compared with the oracle object by object.

8+3 Encode + Reconstruct{0,1,2} of 4096 objects, each 4 KiB or 1 MiB (p =
0.5, chosen by the splitmix byte stream exactly as bench.config4 does), laid
out as an object plan (data arena + parity arena, hbec_plan_objects) and
coded in one launch per op.  Every object's parity is compared with the CPU
oracle's encode of its data (oracle/gf_oracle.c), and the reconstruct
rebuilds shards 0-2 of every object in place after they are overwritten,
which must give back the data arena byte for byte (the oracle's reconstruct
of a codeword is its data).  Reference: objectserver/ecutils.go:59 (Encode)
and :111 (Reconstruct), README's 4 KB bench shape.
"""
import numpy as np
import pytest
import torch

from hummingbird_amd import batch as B
from hummingbird_amd import reedsolomon as RS
from oracle import coracle as CO

pytestmark = pytest.mark.gpu
MiB = 1 << 20


def _mixed_sizes(n):
    flags = torch.empty((1, n), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(flags, n)
    return [MiB if int(b) & 1 else 4096 for b in flags.cpu()[0].tolist()]


def _oracle_check(k, m, data_h, parity_h, dl, pl):
    """Group the objects by size and encode each group on the CPU oracle."""
    by_size = {}
    for i, ((o, s), po) in enumerate(zip(dl, pl)):
        by_size.setdefault(s, []).append((i, o, po))
    for s, items in by_size.items():
        objs = np.stack([data_h[o:o + k * s] for _, o, _ in items])
        want, _ = CO.encode_batch(k, m, objs, threads=CO.cpu_threads())
        got = np.stack([parity_h[po:po + m * s] for _, _, po in items])
        if not np.array_equal(got, want):
            bad = int(np.nonzero((got != want).any(axis=1))[0][0])
            raise AssertionError(f"object {items[bad][0]} (S = {s}) differs from the oracle")
    return sum(len(v) for v in by_size.values())


def test_config4_full_mixed_objects_oracle():
    torch.cuda.set_device(0)
    k, m, n = 8, 3, 4096
    sizes = _mixed_sizes(n)
    assert 0 < sum(1 for x in sizes if x == MiB) < n  # both classes present
    enc = RS.New(k, m)
    dl, pl, doff, poff = [], [], 0, 0
    for size in sizes:
        s = size // k
        dl.append((doff, s))
        pl.append(poff)
        doff += k * s
        poff += m * s
    data = torch.empty(doff, dtype=torch.uint8, device="cuda")
    parity = torch.full((poff,), 0x5A, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(data.view(1, -1), doff, first=7)
    want = data.clone()
    plan = B.StripePlan(enc, objects=[(data.data_ptr() + o, parity.data_ptr() + po, s)
                                      for (o, s), po in zip(dl, pl)])
    plan.encode()
    torch.cuda.synchronize()
    assert _oracle_check(k, m, data.cpu().numpy(), parity.cpu().numpy(), dl, pl) == n
    # erase shards 0-2 of EVERY object (a mask of the ranges [o, o + 3S)),
    # then rebuild them from the rest
    starts = torch.tensor([o for o, _ in dl], device="cuda", dtype=torch.int64)
    lens = torch.tensor([3 * s for _, s in dl], device="cuda", dtype=torch.int64)
    marks = torch.zeros(doff + 1, dtype=torch.int64, device="cuda")
    marks.index_add_(0, starts, torch.ones_like(starts))
    marks.index_add_(0, starts + lens, -torch.ones_like(starts))
    erase = marks.cumsum(0)[:doff] > 0
    data[erase] = 0xC3
    torch.cuda.synchronize()
    assert not torch.equal(data, want)
    present = [0, 0, 0] + [1] * (k + m - 3)
    plan.reconstruct(present)
    torch.cuda.synchronize()
    assert torch.equal(data, want)
    del plan, data, parity, want
    torch.cuda.empty_cache()
