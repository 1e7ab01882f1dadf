#!/usr/bin/env python3
"""BASELINE.json configs beyond the headline, device-resident, one MI355X.

  config 2: 4+2 encode, 4096 x 1 MiB
  config 3: 4+2 reconstruct, 4096 x 1 MiB, erasures {0,1} {0,4} {4,5} {2,3}
  config 4: 8+3 encode + reconstruct{0,1,2}, 4096 objects of 4 KiB or 1 MiB
            (p = 0.5 each, drawn by splitmix64(seed) per index; one launch per
            op through a stripe plan)
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
    s = size // k
    enc = RS.New(k, m)
    objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, size)
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
    ms = timeit(lambda: B.encode_views(enc, views, n, s))
    line(f"{k}+{m} encode {n}x{size}", n * (k + m) * s, ms, kernel=B.kernel_info(k, m, s)["kind"])
    for i in [0, n // 2, n - 1]:
        o, p = objs[i].cpu().numpy(), par[i].cpu().numpy()
        assert U.verify_shards(enc, [o[j * s:(j + 1) * s] for j in range(k)] + [p[r * s:(r + 1) * s] for r in range(m)])
    # Verify (read-only: k+m shards read per object, one flag word written)
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    ms = timeit(lambda: B.verify_views(enc, views, n, s, flags))
    assert int(flags.sum()) == 0
    par[n // 3, 5] ^= 1
    flags.zero_()
    B.verify_views(enc, views, n, s, flags)
    torch.cuda.synchronize()
    assert flags.nonzero().flatten().tolist() == [n // 3]
    par[n // 3, 5] ^= 1
    line(f"{k}+{m} verify {n}x{size}", n * (k + m) * s, ms, bound="HBM read")
    for miss in patterns:
        out = torch.empty((n, len(miss) * s), dtype=torch.uint8, device="cuda")
        rv = list(views)
        for slot, i in enumerate(miss):
            rv[i] = (out.data_ptr() + slot * s, out.stride(0))
        present = [0 if i in miss else 1 for i in range(k + m)]
        ms = timeit(lambda: B.reconstruct_views(enc, rv, present, n, s))
        torch.cuda.synchronize()
        for slot, i in enumerate(miss):
            src = objs[:, i * s:(i + 1) * s] if i < k else par[:, (i - k) * s:(i - k + 1) * s]
            assert torch.equal(out[:, slot * s:(slot + 1) * s], src), miss
        line(f"{k}+{m} reconstruct{set(miss)} {n}x{size}", n * (k + len(miss)) * s, ms)


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


def mixed_8_3(n=4096):
    k, m = 8, 3
    flags = U.splitmix_bytes(n)
    sizes = [MiB if b & 1 else 4096 for b in flags]
    layout, off = [], 0
    for size in sizes:
        s = size // k
        layout.append((off, s))
        off += (k + m) * s
    pool = torch.empty(off, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(pool.view(1, -1), off)
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, [(pool.data_ptr() + o, s) for o, s in layout])
    enc_bytes = sum((k + m) * s for _, s in layout)
    ms = timeit(plan.encode)
    n_big = sum(1 for x in sizes if x == MiB)
    line(f"8+3 encode mixed 4KiB/1MiB x{n} (plan)", enc_bytes, ms, n_1MiB=n_big, n_4KiB=n - n_big,
         plan=plan.info())
    host = pool.cpu().numpy()
    for i in [0, 1, 2, n - 1] + [j for j in range(n) if sizes[j] == 4096][:3]:
        o, s = layout[i]
        assert U.verify_stripe(enc, host[o:o + (k + m) * s])
    ref = pool.clone()
    miss = (0, 1, 2)
    present = [0 if i in miss else 1 for i in range(k + m)]
    ms = timeit(lambda: plan.reconstruct(present))
    assert torch.equal(pool, ref)  # rebuilt in place == original
    rec_bytes = sum((k + len(miss)) * s for _, s in layout)
    line(f"8+3 reconstruct{{0,1,2}} mixed 4KiB/1MiB x{n} (plan)", rec_bytes, ms)
    t_enc = timeit(plan.encode, reps=5)
    t_rec = timeit(lambda: plan.reconstruct(present), reps=5)
    line(f"8+3 encode+reconstruct mixed x{n} (config 4)", enc_bytes + rec_bytes, t_enc + t_rec)


def mixed_8_3_objects(n=4096):
    """Config 4 over an object plan: objects back to back in a data arena,
    parity back to back in a parity arena (hbec_plan_objects)."""
    k, m = 8, 3
    flags = U.splitmix_bytes(n)
    sizes = [MiB if b & 1 else 4096 for b in flags]
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
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, objects=[(data.data_ptr() + o, parity.data_ptr() + po, s)
                                      for (o, s), po in zip(dl, pl)])
    enc_bytes = sum((k + m) * s for _, s in dl)
    ms = timeit(plan.encode)
    line(f"8+3 encode mixed 4KiB/1MiB x{n} (object plan)", enc_bytes, ms, plan=plan.info())
    hd, hp = data.cpu().numpy(), parity.cpu().numpy()
    for i in [0, 1, 2, n - 1] + [j for j in range(n) if sizes[j] == 4096][:3]:
        (o, s), po = dl[i], pl[i]
        assert U.verify_shards(enc, [hd[o + j * s:o + (j + 1) * s] for j in range(k)] +
                               [hp[po + r * s:po + (r + 1) * s] for r in range(m)])
    ref = data.clone()
    miss = (0, 1, 2)
    present = [0 if i in miss else 1 for i in range(k + m)]
    ms = timeit(lambda: plan.reconstruct(present))
    assert torch.equal(data, ref)  # rebuilt in place == original
    rec_bytes = sum((k + len(miss)) * s for _, s in dl)
    line(f"8+3 reconstruct{{0,1,2}} mixed 4KiB/1MiB x{n} (object plan)", rec_bytes, ms)
    t_enc = timeit(plan.encode, reps=5)
    t_rec = timeit(lambda: plan.reconstruct(present), reps=5)
    line(f"8+3 encode+reconstruct mixed x{n} (config 4, object plan)", enc_bytes + rec_bytes, t_enc + t_rec)


def mixed_8_3_size_classes(n=4096):
    """Config 4 with size-classed arenas: the batch's objects are placed by
    size class, each class as a strided batch (objs [n_c][L_c] + parity
    [n_c][m*S_c], the layout of the headline): 1 MiB objects run on the
    pipelined kernel, 4 KiB objects on the short-shard kernel.  Two launches
    per op, timed together."""
    k, m = 8, 3
    flags = U.splitmix_bytes(n)
    sizes = [MiB if b & 1 else 4096 for b in flags]
    enc = RS.New(k, m)
    classes = []
    for size in (MiB, 4096):
        idx = [i for i, x in enumerate(sizes) if x == size]
        s = size // k
        objs = torch.empty((len(idx), size), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(objs, size)
        par = torch.empty((len(idx), m * s), dtype=torch.uint8, device="cuda")
        views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
        classes.append((len(idx), s, objs, par, views))
    miss = (0, 1, 2)
    present = [0 if i in miss else 1 for i in range(k + m)]

    def encode():
        for cnt, s, _, _, v in classes:
            B.encode_views(enc, v, cnt, s)

    def reconstruct():
        for cnt, s, _, _, v in classes:
            B.reconstruct_views(enc, v, present, cnt, s)

    encode()
    torch.cuda.synchronize()
    for cnt, s, objs, par, _ in classes:
        ho, hp = objs[:3].cpu().numpy(), par[:3].cpu().numpy()
        for i in range(3):
            assert U.verify_shards(enc, [ho[i, j * s:(j + 1) * s] for j in range(k)] +
                                   [hp[i, r * s:(r + 1) * s] for r in range(m)])
    refs = [objs.clone() for _, _, objs, _, _ in classes]
    enc_bytes = sum(cnt * (k + m) * s for cnt, s, _, _, _ in classes)
    rec_bytes = sum(cnt * (k + len(miss)) * s for cnt, s, _, _, _ in classes)
    ms = timeit(encode)
    line(f"8+3 encode mixed 4KiB/1MiB x{n} (size-classed arenas)", enc_bytes, ms,
         n_1MiB=classes[0][0], n_4KiB=classes[1][0])
    ms = timeit(reconstruct)
    for ref, (_, _, objs, _, _) in zip(refs, classes):
        assert torch.equal(objs, ref)  # rebuilt in place == original
    line(f"8+3 reconstruct{{0,1,2}} mixed 4KiB/1MiB x{n} (size-classed arenas)", rec_bytes, ms)
    t_enc = timeit(encode, reps=5)
    t_rec = timeit(reconstruct, reps=5)
    line(f"8+3 encode+reconstruct mixed x{n} (config 4, size-classed arenas)", enc_bytes + rec_bytes, t_enc + t_rec)


def main():
    torch.cuda.set_device(0)
    uniform(4, 2, 4096, MiB, [(0, 1), (0, 4), (4, 5), (2, 3)])
    uniform(8, 3, 4096, MiB, [(0, 1, 2)])
    uniform_plan(4, 2, 4096, MiB)
    uniform_plan(8, 3, 4096, MiB)
    mixed_8_3()
    mixed_8_3_objects()
    mixed_8_3_size_classes()


if __name__ == "__main__":
    main()
