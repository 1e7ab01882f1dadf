#!/usr/bin/env python3
"""Headline workload (4+2, 4096 x 1 MiB: encode + reconstruct{0,1}) on buffers
placed different ways, timed interleaved in one process:
  separate - objs / parity / rebuilt as three torch allocations (bench.py)
  arena8   - one 8 GiB allocation carved into the three
  arenaXX  - one XX GiB allocation, the three carved from its start
Prints per variant: median encode / reconstruct ms and fraction of 8 TB/s."""
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

k, m, n, size = 4, 2, 4096, 1 << 20
s = size // k
GiB = 1 << 30


def carve(pool, off, rows, cols):
    return pool[off:off + rows * cols].view(rows, cols), off + rows * cols


def make(kind):
    if kind == "separate":
        objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
        par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
        reb = torch.empty((n, 2 * s), dtype=torch.uint8, device="cuda")
        keep = [objs, par, reb]
    else:
        gib = int(kind[5:])
        pool = torch.empty(gib * GiB, dtype=torch.uint8, device="cuda")
        objs, off = carve(pool, 0, n, size)
        par, off = carve(pool, off, n, m * s)
        reb, off = carve(pool, off, n, 2 * s)
        keep = [pool]
    B.fill_splitmix(objs, size)
    enc = RS.New(k, m)
    ev = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
    rv = [(reb.data_ptr(), reb.stride(0)), (reb.data_ptr() + s, reb.stride(0))] + ev[2:]
    present = [0, 0, 1, 1, 1, 1]
    return keep, (lambda: B.encode_views(enc, ev, n, s)), (lambda: B.reconstruct_views(enc, rv, present, n, s)), (objs, reb)


def main():
    torch.cuda.set_device(0)
    kinds = sys.argv[1:] or ["separate", "arena8", "arena16", "arena64", "arena128"]
    sets = {kd: make(kd) for kd in kinds}
    t = {kd: ([], []) for kd in kinds}
    for kd, (_, e, r, _) in sets.items():
        e(); r()
    for rnd in range(8):
        for kd in (kinds if rnd % 2 == 0 else kinds[::-1]):
            _, e, r, _ = sets[kd]
            for _ in range(3):
                a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                a.record(); e(); b.record(); r(); c.record()
                torch.cuda.synchronize()
                t[kd][0].append(a.elapsed_time(b))
                t[kd][1].append(b.elapsed_time(c))
    byt = n * (k + m) * s
    for kd in kinds:
        objs, reb = sets[kd][3]
        ok = bool(torch.equal(reb, objs[:, :2 * s]))
        te, tr = statistics.median(t[kd][0]), statistics.median(t[kd][1])
        print(json.dumps({"variant": kd, "enc_ms": round(te, 4), "rec_ms": round(tr, 4),
                          "frac": round(2 * byt / ((te + tr) * 1e-3) / 1e9 / 8000, 4), "rebuilt_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
