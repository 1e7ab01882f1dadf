#!/usr/bin/env python3
"""BASELINE configs[4] at G=1 (65 536 x 1 MiB 4+2, 96 GiB resident): why is
the whole-partition encode slower per byte than the 4096-object headline?
Times, on the SAME buffers, interleaved:
  whole   - one hbec_encode_batch over all 65 536 objects
  chunked - 16 launches of 4096 objects each (same bytes)
  first4k - one launch over the first 4096 objects only (x16 for the total)
  last4k  - one launch over the last 4096 objects only
Prints one JSON line per case (ms for the whole partition, fraction of 8 TB/s)."""
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


def main():
    torch.cuda.set_device(0)
    k, m, size = 4, 2, 1 << 20
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    chunk = 4096
    s = size // k
    enc = RS.New(k, m)
    objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, size)

    def part(a, b):
        B.encode_objects(enc, objs[a:b], par[a:b], s)

    cases = {
        "whole": lambda: part(0, n),
        "chunked": lambda: [part(a, min(n, a + chunk)) for a in range(0, n, chunk)],
        "first4k": lambda: part(0, chunk),
        "last4k": lambda: part(n - chunk, n),
    }
    scale = {"whole": 1, "chunked": 1, "first4k": n // chunk, "last4k": n // chunk}
    t = {c: [] for c in cases}
    for f in cases.values():
        f()
    for rnd in range(6):
        for c in (list(cases) if rnd % 2 == 0 else list(cases)[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            cases[c]()
            e1.record()
            torch.cuda.synchronize()
            t[c].append(e0.elapsed_time(e1) * scale[c])
    nbytes = n * (k + m) * s
    for c, v in t.items():
        ms = statistics.median(v)
        print(json.dumps({"case": c, "objects": n, "ms_whole_partition": round(ms, 3),
                          "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 1e9 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
