#!/usr/bin/env python3
"""A/B of gf_odd (odd.hip) build variants on odd shard lengths: one variant
library per process (HBEC_LIB), processes alternated as scripts/ab_odd.sh does.

    python scripts/tune_odd.py build v1,v2        # CPU: tune_build/odd_<v>/libhbec.so
    HBEC_LIB=tune_build/odd_<v>/libhbec.so python scripts/tune_odd.py run <v> [round]

Prints one JSON line per (variant, shape): median ms and % of 8 TB/s for
Encode, Verify and (databuf shapes) Reconstruct of two shards; every result
is checked by Verify on the GPU.
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

# variants override the odd-kernel constants of tuning.h (-D), built with
# HBEC_TUNE=1 so runtime tune_knob variables (HBEC_ODD_BPC, ...) are read
VARIANTS = {
    "base": [],
    "umid2": ["HBEC_ODD_U_MID=2"],
    "planu1": ["HBEC_ODD_PLAN_U=1"],
    "rec16": ["HBEC_ODD_REC_MINKR=16"],
    "lds5": ["HBEC_ODD_LDS_MINK=5"],
}

MiB = 1 << 20
SHAPES = [(4, 2, MiB - 4, "databuf"), (4, 2, MiB - 4, "split"), (4, 2, 1000001, "databuf"), (8, 3, MiB - 8, "databuf"),
          (6, 3, MiB, "databuf"), (10, 4, MiB, "databuf"), (12, 4, 12 * 87392 - 5, "databuf")]


def build(names=None):
    from hummingbird_amd import build as Bd

    for name, defs in VARIANTS.items():
        if names and name not in names:
            continue
        out = ROOT / "tune_build" / f"odd_{name}"
        Bd.build(defs=["HBEC_TUNE=1"] + defs, lib=out / "libhbec.so", objdir=out / "obj", verbose=False)
        print("built", out, flush=True)


def run(label, rnd=0, n=2048):
    import torch

    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS

    torch.cuda.set_device(0)

    def timeit(fn, reps=15):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts)

    # clock settle
    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for _ in range(200):
        x.add_(1)
    del x
    for k, m, L, layout in SHAPES:
        s = -(-L // k)
        enc = RS.New(k, m)
        if layout == "databuf":
            rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(rows, (k + m) * s)
            views = B.shard_views(rows, k + m, s)
        else:
            objs = torch.empty((n, k * s), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(objs, k * s)
            par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
            views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        nb = n * (k + m) * s
        row = {"variant": label, "round": rnd, "k": k, "m": m, "S": s, "layout": layout}
        ms = timeit(lambda: B.encode_views(enc, views, n, s))
        row["encode"] = round(nb / (ms * 1e-3) / 8e12, 4)
        if layout == "databuf":
            present = [0, 0] + [1] * (k + m - 2)
            ms = timeit(lambda: B.reconstruct_views(enc, views, present, n, s))
            row["reconstruct"] = round(n * (k + 2) * s / (ms * 1e-3) / 8e12, 4)
        ms = timeit(lambda: B.verify_views(enc, views, n, s, flags))
        row["verify"] = round(nb / (ms * 1e-3) / 8e12, 4)
        flags.zero_()
        B.verify_views(enc, views, n, s, flags)
        torch.cuda.synchronize()
        row["ok"] = int(flags.count_nonzero().item()) == 0
        print(json.dumps(row), flush=True)
        del views
        torch.cuda.empty_cache()
    # plans: n ecSplit databufs of 1 MiB - (1..15) B back to back (stripe plan),
    # and k > 8 object plans (data arena + parity arena)
    import numpy as np

    for k, m, uniform in [(4, 2, False), (4, 2, True), (8, 3, False), (10, 4, False)]:
        rng = np.random.default_rng(k * 100 + m)
        layout, off = [], 0
        for _ in range(n):
            s = -(-((1 << 20) - (4 if uniform else int(rng.integers(1, 16)))) // k)
            layout.append((off, s))
            off += (k + m) * s
        pool = torch.empty((1, off), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(pool, off)
        enc = RS.New(k, m)
        plan = B.StripePlan(enc, [(pool.data_ptr() + o, s) for o, s in layout])
        ms = timeit(plan.encode)
        nb = sum((k + m) * s for _, s in layout)
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        for i, (o, s) in enumerate(layout[:64]):
            v = [(pool.data_ptr() + o + j * s, 0) for j in range(k + m)]
            B.verify_views(enc, v, 1, s, flags[i:i + 1])
        torch.cuda.synchronize()
        print(json.dumps({"variant": label, "round": rnd, "k": k, "m": m,
                          "layout": "stripe plan odd" + (" uniform S" if uniform else ""),
                          "encode": round(nb / (ms * 1e-3) / 8e12, 4),
                          "ok": int(flags.count_nonzero().item()) == 0}), flush=True)
        del pool, plan
        torch.cuda.empty_cache()
    for k, m, s in [(10, 4, 104858), (12, 4, 87392)]:
        d = torch.empty((n, k * s), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(d, k * s)
        par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
        enc = RS.New(k, m)
        plan = B.StripePlan(enc, objects=[(d.data_ptr() + i * d.stride(0), par.data_ptr() + i * par.stride(0), s)
                                          for i in range(n)])
        ms = timeit(plan.encode)
        nb = n * (k + m) * s
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.verify_views(enc, B.shard_views(d, k, s) + B.shard_views(par, m, s), n, s, flags)
        torch.cuda.synchronize()
        print(json.dumps({"variant": label, "round": rnd, "k": k, "m": m, "S": s, "layout": "object plan",
                          "encode": round(nb / (ms * 1e-3) / 8e12, 4),
                          "ok": int(flags.count_nonzero().item()) == 0}), flush=True)
        del d, par, plan
        torch.cuda.empty_cache()


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build(sys.argv[2].split(",") if len(sys.argv) > 2 else None)
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "default", int(sys.argv[3]) if len(sys.argv) > 3 else 0)
