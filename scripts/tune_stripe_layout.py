#!/usr/bin/env python3
"""Layout A/B for the headline workload (4+2 @ 1 MiB x 4096, encode +
reconstruct{0,1}), interleaved rounds in one process:

  split   — objs [n][k*S] + parity [n][m*S] + rebuilt [n][2*S] (bench.py until now)
  stripe  — one array [n][(k+m)*S]: ecSplit's databuf layout
            (objectserver/ecutils.go:31-35,55-58); encode writes the parity
            shards into the row, reconstruct rebuilds shards 0,1 in place in
            the row, as ecReconstruct does in its databuf (ecutils.go:94-111)

Prints per-layout median encode / reconstruct ms and % of 8 TB/s.
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402


def main(n=4096, rounds=20, launches=4, k=4, m=2):
    torch.cuda.set_device(0)
    S = (1 << 20) // k
    enc = RS.New(k, m)
    e = min(m, 2)
    present = [0] * e + [1] * (k + m - e)
    # split layout
    objs = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * S)
    par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    reb = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
    sv_enc = B.shard_views(objs, k, S) + B.shard_views(par, m, S)
    sv_rec = list(sv_enc)
    for i in range(e):
        sv_rec[i] = (reb.data_ptr() + i * S, reb.stride(0))
    # stripe layout
    rows = torch.empty((n, (k + m) * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(rows, k * S)
    st_views = B.shard_views(rows, k + m, S)
    lay = {"split": (sv_enc, sv_rec), "stripe": (st_views, st_views)}
    t = {name: {"enc": [], "rec": []} for name in lay}
    for rnd in range(rounds + 1):
        for name, (ve, vr) in (lay.items() if rnd % 2 == 0 else reversed(list(lay.items()))):
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * launches + 1)]
            torch.cuda.synchronize()
            evs[0].record()
            for i in range(launches):
                B.encode_views(enc, ve, n, S)
                evs[2 * i + 1].record()
                B.reconstruct_views(enc, vr, present, n, S)
                evs[2 * i + 2].record()
            torch.cuda.synchronize()
            if rnd:
                for i in range(launches):
                    t[name]["enc"].append(evs[2 * i].elapsed_time(evs[2 * i + 1]))
                    t[name]["rec"].append(evs[2 * i + 1].elapsed_time(evs[2 * i + 2]))
    ok_split = bool(torch.equal(reb, objs[:, :e * S]))
    want = rows[:, :e * S].clone()
    rows[:, :e * S].zero_()
    B.reconstruct_views(enc, st_views, present, n, S)
    ok_stripe = bool(torch.equal(rows[:, :e * S], want)) and bool(torch.equal(rows[:, k * S:], par))
    nbytes = n * (k + m) * S
    for name, ok in (("split", ok_split), ("stripe", ok_stripe)):
        em, rm = statistics.median(t[name]["enc"]), statistics.median(t[name]["rec"])
        print(json.dumps({"layout": name, "k": k, "m": m, "enc_ms": round(em, 4), "rec_ms": round(rm, 4),
                          "enc_frac": round(nbytes / em / 1e6 / 8000, 4),
                          "rec_frac": round(n * (k + e) * S / rm / 1e6 / 8000, 4),
                          "frac": round((nbytes + n * (k + e) * S) / (em + rm) / 1e6 / 8000, 4), "ok": ok}),
              flush=True)




def pitch_sweep(n=4096, k=4, m=2, reps=6, pads=(0, 512, 1024, 2048, 4096, 8192, 16384, 65536), row_pads=(0, 4096)):
    """Stripe layout with shard pitch S + pad (and row pitch (k+m)*pitch +
    row_pad): does spacing the concurrently streamed shards apart help?"""
    torch.cuda.set_device(0)
    S = (1 << 20) // k
    enc = RS.New(k, m)
    e = min(m, 2)
    present = [0] * e + [1] * (k + m - e)
    nbytes = n * (k + m) * S
    big = max(pads)
    pool = torch.empty(n * ((k + m) * (S + big) + max(row_pads)) + (1 << 20), dtype=torch.uint8, device="cuda")
    base = (pool.data_ptr() + 4095) // 4096 * 4096
    for pad in pads:
        for rp in row_pads:
            pitch = S + pad
            row = (k + m) * pitch + rp
            views = [(base + i * pitch, row) for i in range(k + m)]
            assert base + (n - 1) * row + (k + m) * pitch <= pool.data_ptr() + pool.numel()
            te, tr = [], []
            for r in range(reps + 1):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                B.encode_views(enc, views, n, S)
                e1.record()
                B.reconstruct_views(enc, views, present, n, S)
                e2.record()
                torch.cuda.synchronize()
                if r:
                    te.append(e0.elapsed_time(e1))
                    tr.append(e1.elapsed_time(e2))
            em, rm = statistics.median(te), statistics.median(tr)
            print(json.dumps({"sweep": "pitch", "k": k, "m": m, "shard_pad": pad, "row_pad": rp,
                              "enc_ms": round(em, 4), "rec_ms": round(rm, 4),
                              "frac": round((nbytes + n * (k + e) * S) / (em + rm) / 1e6 / 8000, 4)}), flush=True)


def split_sweep(n=4096, k=4, m=2, reps=6, obj_pads=(0, 32768, 65536, 131072, 262144),
                par_offs=(0, 65536, 131072, 196608), par_pads=(0, 65536)):
    """Split layout (objs / parity / rebuilt arrays): object pitch k*S +
    obj_pad, parity and rebuilt bases shifted by par_off, their shard pitch
    S + par_pad.  Which relative placement of the six streams is fastest?"""
    torch.cuda.set_device(0)
    S = (1 << 20) // k
    enc = RS.New(k, m)
    e = min(m, 2)
    present = [0] * e + [1] * (k + m - e)
    nbytes = n * (k + m) * S
    obj_span = n * (k * S + max(obj_pads))
    par_span = n * (m * (S + max(par_pads))) + max(par_offs)
    pool = torch.empty(obj_span + 2 * par_span + (4 << 20), dtype=torch.uint8, device="cuda")
    base = (pool.data_ptr() + (1 << 20) - 1) // (1 << 20) * (1 << 20)
    end = pool.data_ptr() + pool.numel()
    for op in obj_pads:
        for po in par_offs:
            for pp in par_pads:
                orow = k * S + op
                prow = m * (S + pp)
                ob = base
                pb = base + obj_span + po
                rb = pb + par_span
                assert rb + (n - 1) * prow + m * (S + pp) <= end
                ev = [(ob + j * S, orow) for j in range(k)] + [(pb + r * (S + pp), prow) for r in range(m)]
                rv = [(rb + i * (S + pp), prow) for i in range(e)] + ev[e:]
                te, tr = [], []
                for r in range(reps + 1):
                    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                    e0.record()
                    B.encode_views(enc, ev, n, S)
                    e1.record()
                    B.reconstruct_views(enc, rv, present, n, S)
                    e2.record()
                    torch.cuda.synchronize()
                    if r:
                        te.append(e0.elapsed_time(e1))
                        tr.append(e1.elapsed_time(e2))
                em, rm = statistics.median(te), statistics.median(tr)
                print(json.dumps({"sweep": "split", "k": k, "m": m, "obj_pad": op, "par_off": po, "par_pad": pp,
                                  "enc_ms": round(em, 4), "rec_ms": round(rm, 4),
                                  "frac": round((nbytes + n * (k + e) * S) / (em + rm) / 1e6 / 8000, 4)}),
                      flush=True)


def split_ab(n=4096, k=4, m=2, rounds=12, reps=4,
             combos=((0, 0, 0), (0, 65536, 0), (131072, 131072, 0), (0, 131072, 65536), (65536, 131072, 0),
                     (0, 65536 + 4096, 0), (0, 32768, 0))):
    """Interleaved A/B of a few split placements (obj_pad, par_off, par_pad)."""
    torch.cuda.set_device(0)
    S = (1 << 20) // k
    enc = RS.New(k, m)
    e = min(m, 2)
    present = [0] * e + [1] * (k + m - e)
    nbytes = n * (k + m) * S
    mo = max(c[0] for c in combos)
    mp = max(c[2] for c in combos)
    mpo = max(c[1] for c in combos)
    obj_span = n * (k * S + mo)
    par_span = n * m * (S + mp) + mpo
    pool = torch.empty(obj_span + 2 * par_span + (4 << 20), dtype=torch.uint8, device="cuda")
    base = (pool.data_ptr() + (1 << 20) - 1) // (1 << 20) * (1 << 20)
    lay = []
    for op, po, pp in combos:
        orow, prow = k * S + op, m * (S + pp)
        pb = base + obj_span + po
        rb = pb + par_span
        ev = [(base + j * S, orow) for j in range(k)] + [(pb + r * (S + pp), prow) for r in range(m)]
        rv = [(rb + i * (S + pp), prow) for i in range(e)] + ev[e:]
        lay.append(((op, po, pp), ev, rv))
    t = {c: ([], []) for c, _, _ in lay}
    for rnd in range(rounds + 1):
        order = lay if rnd % 2 == 0 else lay[::-1]
        for c, ev, rv in order:
            for r in range(reps):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                B.encode_views(enc, ev, n, S)
                e1.record()
                B.reconstruct_views(enc, rv, present, n, S)
                e2.record()
                torch.cuda.synchronize()
                if rnd:
                    t[c][0].append(e0.elapsed_time(e1))
                    t[c][1].append(e1.elapsed_time(e2))
    for c, _, _ in lay:
        em, rm = statistics.median(t[c][0]), statistics.median(t[c][1])
        print(json.dumps({"sweep": "split_ab", "k": k, "m": m, "obj_pad": c[0], "par_off": c[1], "par_pad": c[2],
                          "enc_ms": round(em, 4), "rec_ms": round(rm, 4),
                          "frac": round((nbytes + n * (k + e) * S) / (em + rm) / 1e6 / 8000, 4)}), flush=True)


def kernels_ab(n=4096, k=4, m=2, rounds=16, reps=3):
    """Interleaved: strided kernel vs stripe-plan kernel vs object-plan kernel,
    on the split and stripe layouts; encode, and reconstruct{0,1} in place."""
    torch.cuda.set_device(0)
    S = (1 << 20) // k
    enc = RS.New(k, m)
    objs = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * S)
    par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    rows = torch.empty((n, (k + m) * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(rows, k * S)
    sv = B.shard_views(objs, k, S) + B.shard_views(par, m, S)
    rv = B.shard_views(rows, k + m, S)
    splan = B.StripePlan(enc, [(rows.data_ptr() + i * rows.stride(0), S) for i in range(n)])
    oplan = B.StripePlan(enc, objects=[(objs.data_ptr() + i * objs.stride(0), par.data_ptr() + i * par.stride(0), S)
                                       for i in range(n)])
    present = [0, 0] + [1] * (k + m - 2)
    reb = torch.empty((n, 2 * S), dtype=torch.uint8, device="cuda")
    sv_reb = [(reb.data_ptr(), reb.stride(0)), (reb.data_ptr() + S, reb.stride(0))] + sv[2:]
    rplan = B.StripePlan(enc, objects=[(objs.data_ptr() + i * objs.stride(0), par.data_ptr() + i * par.stride(0), S)
                                       for i in range(n)])
    cases = {
        "strided_split": lambda: B.encode_views(enc, sv, n, S),
        "strided_stripe": lambda: B.encode_views(enc, rv, n, S),
        "plan_stripe": splan.encode,
        "plan_split": oplan.encode,
        "rec01_strided_split": lambda: B.reconstruct_views(enc, sv, present, n, S),
        "rec01_plan_split": lambda: oplan.reconstruct(present),
        "rec01_plan_stripe": lambda: splan.reconstruct(present),
        "rec01_strided_rebuilt": lambda: B.reconstruct_views(enc, sv_reb, present, n, S),
    }
    t = {c: [] for c in cases}
    names = list(cases)
    for rnd in range(rounds + 1):
        for c in (names if rnd % 2 == 0 else names[::-1]):
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                cases[c]()
                e1.record()
                torch.cuda.synchronize()
                if rnd:
                    t[c].append(e0.elapsed_time(e1))
    ok = bool(torch.equal(par, rows[:, k * S:])) and bool(torch.equal(rows[:, :k * S], objs))
    for c in names:
        ms = statistics.median(t[c])
        nb = n * ((k + 2) if c.startswith("rec01") else (k + m)) * S
        print(json.dumps({"sweep": "kernels", "k": k, "m": m, "case": c, "ms": round(ms, 4),
                          "frac": round(nb / ms / 1e6 / 8000, 4), "ok": ok}), flush=True)


def mixed_ab(n=4096, k=8, m=3, rounds=12, reps=3):
    """Config 4 (8+3, 4 KiB / 1 MiB mixed, p = 0.5) interleaved: stripe plan over
    ecSplit stripes vs object plan over data / parity arenas, and the object
    plan restricted to the big objects or to the small ones."""
    from scripts import _common as U

    torch.cuda.set_device(0)
    MiB = 1 << 20
    flags = U.splitmix_bytes(n)
    sizes = [MiB if b & 1 else 4096 for b in flags]
    enc = RS.New(k, m)
    # stripe layout
    lay, off = [], 0
    for size in sizes:
        s = size // k
        lay.append((off, s))
        off += (k + m) * s
    pool = torch.empty(off, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(pool.view(1, -1), off)
    splan = B.StripePlan(enc, [(pool.data_ptr() + o, s) for o, s in lay])
    # object arenas
    dl, pl, doff, poff = [], [], 0, 0
    for size in sizes:
        s = size // k
        dl.append((doff, s))
        pl.append(poff)
        doff += k * s
        poff += m * s
    data = torch.empty(doff, dtype=torch.uint8, device="cuda")
    par = torch.empty(poff, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(data.view(1, -1), doff)
    objs = [(data.data_ptr() + o, par.data_ptr() + po, s) for (o, s), po in zip(dl, pl)]
    oplan = B.StripePlan(enc, objects=objs)
    big = B.StripePlan(enc, objects=[x for x in objs if x[2] == MiB // k])
    small = B.StripePlan(enc, objects=[x for x in objs if x[2] != MiB // k])
    nb_all = sum((k + m) * s for _, s in lay)
    nb_big = sum((k + m) * x[2] for x in objs if x[2] == MiB // k)
    nb_small = nb_all - nb_big
    cases = {"stripe_plan": (splan.encode, nb_all), "object_plan": (oplan.encode, nb_all),
             "object_plan_big_only": (big.encode, nb_big), "object_plan_small_only": (small.encode, nb_small)}
    t = {c: [] for c in cases}
    names = list(cases)
    for rnd in range(rounds + 1):
        for c in (names if rnd % 2 == 0 else names[::-1]):
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                cases[c][0]()
                e1.record()
                torch.cuda.synchronize()
                if rnd:
                    t[c].append(e0.elapsed_time(e1))
    for c in names:
        ms = statistics.median(t[c])
        print(json.dumps({"sweep": "mixed", "case": c, "ms": round(ms, 4), "bytes": cases[c][1],
                          "frac": round(cases[c][1] / ms / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["mixed"]:
        mixed_ab()
    elif sys.argv[1:2] == ["kernels"]:
        a = [int(x) for x in sys.argv[2:]]
        kernels_ab(k=a[0], m=a[1]) if a else kernels_ab()
    elif sys.argv[1:2] == ["split_ab"]:
        split_ab()
    elif sys.argv[1:2] == ["split"]:
        split_sweep()
    elif sys.argv[1:2] == ["pitch"]:
        a = [int(x) for x in sys.argv[2:]]
        pitch_sweep(k=a[0], m=a[1]) if a else pitch_sweep()
    else:
        a = [int(x) for x in sys.argv[1:]]
        main(k=a[0], m=a[1]) if a else main()
