#!/usr/bin/env python3
"""BASELINE.json configs beyond the headline, device-resident, one MI355X.

  config 2: 4+2 encode, 4096 x 1 MiB
  config 3: 4+2 reconstruct, 4096 x 1 MiB, erasures {0,1} {0,4} {4,5} {2,3}
  config 4: 8+3 encode + reconstruct{0,1,2}, 4096 objects of 4 KiB or 1 MiB
            (p = 0.5 each, drawn by splitmix64(seed) per index) in three
            placements, timed interleaved (config4())
  extra   : 8+3 @ 1 MiB uniform (strided views); Verify of both uniform configs

Algorithmic bytes per object: encode (k+m)*S, reconstruct (k+e)*S.
Prints one JSON line per measurement (GiB/s, GB/s and fraction of 8 TB/s).
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402
from scripts import _common as U  # noqa: E402

MiB = 1 << 20
GiB = float(1 << 30)
PEAK = 8000.0


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def line(name, nbytes, ms, **kw):
    d = {"config": name, "ms": round(ms, 4), "algorithmic_bytes": nbytes,
         "GiB_s": round(nbytes / (ms * 1e-3) / GiB, 1), "GB_s": round(nbytes / (ms * 1e-3) / 1e9, 1),
         "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 1e9 / PEAK, 4)}
    d.update(kw)
    print(json.dumps(d), flush=True)


def uniform(k, m, n, size, patterns):
    """Encode, Verify and Reconstruct (each erasure pattern) of n uniform
    objects, timed interleaved; each op's output is checked afterwards."""
    s = size // k
    enc = RS.New(k, m)
    objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, size)
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
    # Verify (read-only: k+m shards read per object, one flag word written)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    cases = {"encode": lambda: B.encode_views(enc, views, n, s),
             "verify": lambda: B.verify_views(enc, views, n, s, flags)}
    outs = {}
    for miss in patterns:
        out = torch.empty((n, len(miss) * s), dtype=torch.uint8, device="cuda")
        rv = list(views)
        for slot, i in enumerate(miss):
            rv[i] = (out.data_ptr() + slot * s, out.stride(0))
        present = [0 if i in miss else 1 for i in range(k + m)]
        outs[miss] = out
        cases[miss] = (lambda rv=rv, present=present: B.reconstruct_views(enc, rv, present, n, s))
    B.encode_views(enc, views, n, s)  # parity first: verify and reconstruct read it
    t = interleaved(cases)
    for i in [0, n // 2, n - 1]:
        o, q = objs[i].cpu().numpy(), par[i].cpu().numpy()
        assert U.verify_shards(enc, [o[j * s:(j + 1) * s] for j in range(k)] + [q[r * s:(r + 1) * s] for r in range(m)])
    assert int(flags.sum()) == 0
    par[n // 3, 5] ^= 1
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == [n // 3]
    par[n // 3, 5] ^= 1
    for miss, out in outs.items():
        for slot, i in enumerate(miss):
            src = objs[:, i * s:(i + 1) * s] if i < k else par[:, (i - k) * s:(i - k + 1) * s]
            assert torch.equal(out[:, slot * s:(slot + 1) * s], src), miss
    line(f"{k}+{m} encode {n}x{size}", n * (k + m) * s, t["encode"], kernel=B.kernel_info(k, m, s)["kind"])
    line(f"{k}+{m} verify {n}x{size}", n * (k + m) * s, t["verify"], bound="HBM read")
    for miss in patterns:
        line(f"{k}+{m} reconstruct{set(miss)} {n}x{size}", n * (k + len(miss)) * s, t[miss])


def uniform_plan(k, m, n, size):
    """Uniform stripes through a stripe plan (gf_apply_stripes) instead of
    strided views (gf_apply_vec_pipe): isolates the plan kernel's own cost
    from config 4's size mix."""
    s = size // k
    pool = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(pool, (k + m) * s)
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, [(pool.data_ptr() + i * pool.stride(0), s) for i in range(n)])
    ms = timeit(plan.encode)
    line(f"{k}+{m} encode {n}x{size} (plan, uniform)", n * (k + m) * s, ms, plan=plan.info())


def interleaved(cases, rounds=8, reps=3):
    """Median ms per case, cases run in alternating order each round, so clock
    and power drift over a long script hit every case alike."""
    names = list(cases)
    for f in cases.values():  # warm
        f()
    t = {c: [] for c in names}
    for rnd in range(rounds):
        for c in (names if rnd % 2 == 0 else names[::-1]):
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                cases[c]()
                e1.record()
                torch.cuda.synchronize()
                t[c].append(e0.elapsed_time(e1))
    return {c: statistics.median(v) for c, v in t.items()}


def config4(n=4096):
    """Config 4: 8+3 encode + reconstruct{0,1,2} of n objects of 4 KiB or 1 MiB
    (p = 0.5 each, drawn by splitmix64(seed) per index), in three placements,
    timed interleaved:
      stripes  - ecSplit databufs back to back (stripe plan, one launch per op)
      objects  - a data arena + a parity arena (object plan, one launch per op)
      classes  - size-classed strided batches (two launches per op)"""
    k, m = 8, 3
    miss = (0, 1, 2)
    present = [0 if i in miss else 1 for i in range(k + m)]
    flags = U.splitmix_bytes(n)
    sizes = [MiB if b & 1 else 4096 for b in flags]
    enc = RS.New(k, m)
    # stripes
    lay, off = [], 0
    for size in sizes:
        s = size // k
        lay.append((off, s))
        off += (k + m) * s
    pool = torch.empty(off, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(pool.view(1, -1), off)
    splan = B.StripePlan(enc, [(pool.data_ptr() + o, s) for o, s in lay])
    # objects
    dl, pl, doff, poff = [], [], 0, 0
    for size in sizes:
        s = size // k
        dl.append((doff, s))
        pl.append(poff)
        doff += k * s
        poff += m * s
    data = torch.empty(doff, dtype=torch.uint8, device="cuda")
    parity = torch.empty(poff, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(data.view(1, -1), doff)
    oplan = B.StripePlan(enc, objects=[(data.data_ptr() + o, parity.data_ptr() + po, s)
                                       for (o, s), po in zip(dl, pl)])
    # size classes
    classes = []
    for size in (MiB, 4096):
        cnt = sum(1 for x in sizes if x == size)
        s = size // k
        objs = torch.empty((cnt, size), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(objs, size)
        par = torch.empty((cnt, m * s), dtype=torch.uint8, device="cuda")
        classes.append((cnt, s, objs, par, B.shard_views(objs, k, s) + B.shard_views(par, m, s)))

    def cls_encode():
        for cnt, s, _, _, v in classes:
            B.encode_views(enc, v, cnt, s)

    def cls_reconstruct():
        for cnt, s, _, _, v in classes:
            B.reconstruct_views(enc, v, present, cnt, s)

    t = interleaved({
        "stripes_enc": splan.encode, "stripes_rec": lambda: splan.reconstruct(present),
        "objects_enc": oplan.encode, "objects_rec": lambda: oplan.reconstruct(present),
        "classes_enc": cls_encode, "classes_rec": cls_reconstruct,
    })
    # self-checks: parity verifies, and the in-place rebuilds reproduced the data
    hp, hd, hpar = pool.cpu().numpy(), data.cpu().numpy(), parity.cpu().numpy()
    for i in [0, 1, 2, n - 1] + [j for j in range(n) if sizes[j] == 4096][:3]:
        o, s = lay[i]
        assert U.verify_stripe(enc, hp[o:o + (k + m) * s])
        (o, s), po = dl[i], pl[i]
        assert U.verify_shards(enc, [hd[o + j * s:o + (j + 1) * s] for j in range(k)] +
                               [hpar[po + r * s:po + (r + 1) * s] for r in range(m)])
    for cnt, s, objs, par, _ in classes:
        ho, hq = objs[:2].cpu().numpy(), par[:2].cpu().numpy()
        for i in range(2):
            assert U.verify_shards(enc, [ho[i, j * s:(j + 1) * s] for j in range(k)] +
                                   [hq[i, r * s:(r + 1) * s] for r in range(m)])
    enc_bytes = sum((k + m) * s for _, s in lay)
    rec_bytes = sum((k + len(miss)) * s for _, s in lay)
    n_big = sum(1 for x in sizes if x == MiB)
    for name, what in (("stripes", "stripe plan, ecSplit databufs"), ("objects", "object plan, data + parity arenas"),
                       ("classes", "size-classed strided batches, 2 launches per op")):
        line(f"8+3 encode mixed 4KiB/1MiB x{n} ({what})", enc_bytes, t[name + "_enc"], n_1MiB=n_big, n_4KiB=n - n_big)
        line(f"8+3 reconstruct{{0,1,2}} mixed 4KiB/1MiB x{n} ({what})", rec_bytes, t[name + "_rec"])
        line(f"8+3 encode+reconstruct mixed x{n} (config 4, {what})", enc_bytes + rec_bytes,
             t[name + "_enc"] + t[name + "_rec"])


def main():
    torch.cuda.set_device(0)
    uniform(4, 2, 4096, MiB, [(0, 1), (0, 4), (4, 5), (2, 3)])
    uniform(8, 3, 4096, MiB, [(0, 1, 2)])
    uniform_plan(4, 2, 4096, MiB)
    uniform_plan(8, 3, 4096, MiB)
    config4()


if __name__ == "__main__":
    main()
