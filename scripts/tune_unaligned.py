#!/usr/bin/env python3
"""A/B of gf_apply_unaligned's knobs (windows per wave tile, source-dword
selection) on odd shard lengths, one variant library per process.

    python scripts/tune_unaligned.py build [v1,v2]   # CPU: tune_build/unal_*/libhbec.so
    for v in ...; do HBEC_LIB=tune_build/unal_$v/libhbec.so python scripts/tune_unaligned.py run $v; done

Prints one JSON line per (variant, shape, round): median ms and % of 8 TB/s.
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

VARIANTS = {
    "base": [],  # shipped: U = 4, single load + lane shuffle, v_cndmask selection
    "twoload": ["HBEC_UNALIGNED_SHFL=0"],
    "shflu2": ["HBEC_UNALIGNED_U=2"],
}
# third sweep (profiles/r02_tune_stream_clamp_rejected.jsonl): clamped loads in
# the streaming kernel (K > 8, aligned) instead of loads under branches: equal
# within 1 %, not adopted.
# second sweep (profiles/r02_tune_unaligned_shfl.jsonl) ran with U = 2, two
# loads, v_cndmask as base: shfl, shflu4 (now shipped), u4sw, u8.
# first sweep (profiles/r02_tune_unaligned.jsonl) ran with the defaults U = 4
# and the uniform switch: base = u4 switch, sel, u2, u8, u2sel, u8sel.

SHAPES = [(4, 2, (1 << 20) - 4), (8, 3, (1 << 20) - 8), (6, 3, 1 << 20), (10, 4, 1 << 20),
          (10, 4, 10 * 104864), (12, 4, 12 * 87392), (16, 4, 1 << 20)]  # the last three: aligned, streaming kernel


def build(names=None):
    from hummingbird_amd import build as Bd

    for name, defs in VARIANTS.items():
        if names and name not in names:
            continue
        out = ROOT / "tune_build" / f"unal_{name}"
        Bd.build(defs=defs, lib=out / "libhbec.so", objdir=out / "obj", verbose=False)
        print("built", out, flush=True)


def run(label, n=2048, rounds=3):
    import torch

    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS

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

    work = []
    for k, m, L in SHAPES:
        s = -(-L // k)
        rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(rows, (k + m) * s)
        enc = RS.New(k, m)
        views = B.shard_views(rows, k + m, s)
        work.append((f"{k}+{m} S={s} databuf encode", n * (k + m) * s,
                     lambda enc=enc, views=views, s=s: B.encode_views(enc, views, n, s), rows))
    for r in range(rounds):
        for name, nbytes, fn, _ in work:
            ms = timeit(fn)
            print(json.dumps({"variant": label, "work": name, "round": r, "ms": round(ms, 4),
                              "frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build(sys.argv[2].split(",") if len(sys.argv) > 2 else None)
    else:
        run(sys.argv[2] if len(sys.argv) > 2 else "default")
