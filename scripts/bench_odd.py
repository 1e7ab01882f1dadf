#!/usr/bin/env python3
"""Device-resident Encode / Reconstruct of shard lengths that are not a
multiple of 16 B (objects of arbitrary size: ecSplit's S = ceil(len / k),
objectserver/ecutils.go:14-24), next to the aligned shape of the same size,
and wide policies (k > 8).  One JSON line per shape: ms, % of 8 TB/s, kernel
kind, and a Verify self-check (scripts/_common.py: no oracle here).

    python scripts/bench_odd.py [n_objects]
"""
from __future__ import annotations

import json
import os
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402

PEAK = 8000.0


def timeit(fn, reps=7, warm=2):
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


def shape(k, m, n, obj_len, layout):
    """layout 'split': objects [n, k*S] + parity [n, m*S];
    'databuf': ecSplit rows [n, (k+m)*S] (shard i at i*S)."""
    s = -(-obj_len // k)
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
    ms = timeit(lambda: B.encode_views(enc, views, n, s))
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.verify_views(enc, views, n, s, flags)
    ok = int(flags.count_nonzero().item()) == 0
    vms = timeit(lambda: B.verify_views(enc, views, n, s, flags))  # read-only: (k+m)*S read
    nb = n * (k + m) * s
    info = B.kernel_info(k, m, s) if k <= 16 else {}
    print(json.dumps({"k": k, "m": m, "n": n, "obj_len": obj_len, "shard_len": s, "layout": layout,
                      "encode_ms": round(ms, 4), "GB_s": round(nb / ms / 1e6, 1),
                      "frac": round(nb / ms / 1e6 / PEAK, 4), "kind": info.get("kind"),
                      "verify_ms": round(vms, 4), "verify_frac": round(nb / vms / 1e6 / PEAK, 4),
                      "verify_ok": ok}), flush=True)


def plan_shape(k, m, n, odd):
    """A stripe plan of n ecSplit databufs back to back, objects of 1 MiB
    (odd=False) or 1 MiB - (1..15) B (odd=True: S % 16 != 0 for most, bases
    at arbitrary offsets), as a batched stabilizer would hand them over."""
    import numpy as np

    rng = np.random.default_rng(k * 100 + m)
    layout, off = [], 0
    for _ in range(n):
        size = (1 << 20) - (int(rng.integers(1, 16)) if odd else 0)
        s = -(-size // k)
        layout.append((off, s))
        off += (k + m) * s
    pool = torch.empty((1, off), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(pool, off)
    enc = RS.New(k, m)
    plan = B.StripePlan(enc, [(pool.data_ptr() + o, s) for o, s in layout])
    ms = timeit(plan.encode)
    nb = sum((k + m) * s for _, s in layout)
    info = plan.info()
    print(json.dumps({"k": k, "m": m, "n": n, "layout": "stripe plan, " + ("odd sizes" if odd else "1 MiB"),
                      "encode_ms": round(ms, 4), "GB_s": round(nb / ms / 1e6, 1),
                      "frac": round(nb / ms / 1e6 / PEAK, 4), "n_fallback": info["n_fallback"]}), flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    torch.cuda.set_device(0)
    MiB = 1 << 20
    for k, m, L in [(4, 2, MiB), (4, 2, MiB - 4), (4, 2, 1000001), (8, 3, MiB - 8), (6, 3, MiB),
                    (10, 4, MiB), (10, 4, 10 * 104864), (12, 4, 12 * 87392), (16, 4, MiB), (17, 3, 17 * 61696)]:
        for layout in ("split", "databuf"):
            shape(k, m, n, L, layout)
    for k, m in [(4, 2), (8, 3), (10, 4)]:
        for odd in (False, True):
            plan_shape(k, m, n, odd)


if __name__ == "__main__":
    main()
