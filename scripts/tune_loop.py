#!/usr/bin/env python3
"""How the headline's launch sequence affects the kernel's rate (same buffers,
interleaved rounds):
  pairs_b2b    - 20 x (encode, reconstruct{0,1}) back to back (bench.py's loop)
  pairs_sync   - the same with a device sync after every pair
  enc_b2b      - 20 encodes back to back
  rec_b2b      - 20 reconstructs back to back
Per-launch HIP-event times, median; fraction of 8 TB/s."""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    torch.cuda.set_device(0)
    w = bench.Workload(4, 2, 4096, 1 << 20, 0, (0, 1))
    steps = 20

    def run(kind):
        enc_t, rec_t = [], []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * steps + 1)]
        torch.cuda.synchronize()
        ev[0].record()
        for i in range(steps):
            if kind in ("pairs_b2b", "pairs_sync", "enc_b2b"):
                w.encode()
            else:
                w.reconstruct()
            ev[2 * i + 1].record()
            if kind in ("pairs_b2b", "pairs_sync"):
                w.reconstruct()
            ev[2 * i + 2].record()
            if kind == "pairs_sync":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        for i in range(steps):
            a = ev[2 * i].elapsed_time(ev[2 * i + 1])
            b = ev[2 * i + 1].elapsed_time(ev[2 * i + 2])
            if kind == "pairs_b2b" or kind == "pairs_sync":
                enc_t.append(a)
                rec_t.append(b)
            elif kind == "enc_b2b":
                enc_t.append(a + b)  # b ~ 0: the second event follows immediately
            else:
                rec_t.append(a + b)
        return enc_t, rec_t

    kinds = ["pairs_b2b", "pairs_sync", "enc_b2b", "rec_b2b"]
    acc = {k: ([], []) for k in kinds}
    for k in kinds:
        run(k)
    for rnd in range(6):
        for k in (kinds if rnd % 2 == 0 else kinds[::-1]):
            e, r = run(k)
            acc[k][0].extend(e)
            acc[k][1].extend(r)
    nbytes = w.enc_bytes
    for k in kinds:
        e, r = acc[k]
        row = {"variant": k}
        if e:
            row["enc_ms"] = round(statistics.median(e), 4)
            row["enc_frac"] = round(nbytes / (row["enc_ms"] * 1e-3) / 1e9 / 8000, 4)
        if r:
            row["rec_ms"] = round(statistics.median(r), 4)
            row["rec_frac"] = round(nbytes / (row["rec_ms"] * 1e-3) / 1e9 / 8000, 4)
        print(json.dumps(row), flush=True)
    assert w.verify()


if __name__ == "__main__":
    main()
