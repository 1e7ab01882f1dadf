#!/usr/bin/env python3
"""A/B of the stripe-plan and verify kernels' tile depth / grid (one variant
per process: HBEC_LIB selects the variant library, env the grid override).

    python scripts/tune_plan.py build [v1,v2]  # CPU side: tune_build/plan_*/libhbec.so
    bash   scripts/tune_plan.sh              # GPU side: every variant, 3 rounds

Prints one JSON line per (variant, workload): median ms and % of 8 TB/s.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

VARIANTS = {
    "base": [],
    "st24": ["HBEC_STRIPE_LOADS=24"],
    "st8": ["HBEC_STRIPE_LOADS=8"],
    "st16": ["HBEC_STRIPE_LOADS=16"],
    "st32": ["HBEC_STRIPE_LOADS=32"],
    "vf8": ["HBEC_VERIFY_LOADS=8"],
    "vf16": ["HBEC_VERIFY_LOADS=16"],
    "vf32": ["HBEC_VERIFY_LOADS=32"],
    "xcd0": ["HBEC_XCD_MAP=0"],
    # stripes kernel pacing (round 2): barrier per tile on (default) / off, s_sleep
    "stnb": ["HBEC_STRIPES_BARRIER=0"],
    "stb_s4": ["HBEC_STRIPES_SLEEP=4"],
    "stb_s8": ["HBEC_STRIPES_SLEEP=8"],
    "stnb_s8": ["HBEC_STRIPES_BARRIER=0", "HBEC_STRIPES_SLEEP=8"],
}


def build(names=None):
    from hummingbird_amd import build as Bd

    for name, defs in VARIANTS.items():
        if names and name not in names:
            continue
        out = ROOT / "tune_build" / f"plan_{name}"
        Bd.build(defs=defs, lib=out / "libhbec.so", objdir=out / "obj", verbose=False)
        print("built", out, flush=True)


def run(label):
    import torch

    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS
    from scripts import _common as U

    MiB = 1 << 20
    torch.cuda.set_device(0)

    def timeit(fn, reps=9):
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

    def emit(work, nbytes, ms):
        print(json.dumps({"variant": label, "work": work, "ms": round(ms, 4),
                          "frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)

    for k, m in ((4, 2), (8, 3)):
        s = MiB // k
        n = 4096
        pool = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(pool, (k + m) * s)
        enc = RS.New(k, m)
        plan = B.StripePlan(enc, [(pool.data_ptr() + i * pool.stride(0), s) for i in range(n)])
        emit(f"{k}+{m} plan encode uniform", n * (k + m) * s, timeit(plan.encode))
        views = B.shard_views(pool, k + m, s)
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        emit(f"{k}+{m} verify", n * (k + m) * s, timeit(lambda: B.verify_views(enc, views, n, s, flags)))
        assert int(flags.sum()) == 0
        del pool, plan
    # config 4 mix
    k, m, n = 8, 3, 4096
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
    emit("8+3 mixed encode (config 4)", sum((k + m) * s for _, s in layout), timeit(plan.encode))
    present = [0, 0, 0] + [1] * 8
    emit("8+3 mixed reconstruct{0,1,2} (config 4)", sum((k + 3) * s for _, s in layout),
         timeit(lambda: plan.reconstruct(present)))


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build(sys.argv[2].split(",") if len(sys.argv) > 2 else None)
    else:
        run(os.environ.get("TUNE_LABEL", "base"))
