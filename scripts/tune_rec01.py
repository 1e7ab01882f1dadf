#!/usr/bin/env python3
"""Placement probe for 4+2 Reconstruct{0,1} vs {2,3}.

Both read two data shards + both parity shards and write two shards; {0,1}
reads the second half of each 1 MiB object row, {2,3} the first.  Cases, timed
interleaved on the same buffers (median of 8 rounds x 5 launches):
  rec01        survivors 2,3 in the object rows, out -> rebuilt
  rec23        survivors 0,1 in the object rows, out -> rebuilt
  rec01_half   survivors 2,3 copied to their own [n, 512 KiB] array (row offset 0)
  rec01_shift  as rec01, rebuilt written 256 KiB further into a padded array
  rec01_inplace as rec01, rebuilt written into the object rows' slots 0,1
"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402

MiB = 1 << 20


def main(n=4096, rounds=8, reps=5):
    torch.cuda.set_device(0)
    k, m, s = 4, 2, MiB // 4
    enc = RS.New(k, m)
    objs = torch.empty((n, MiB), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, MiB)
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    B.encode_objects(enc, objs, par, s)
    rebuilt = torch.empty((n, 2 * s), dtype=torch.uint8, device="cuda")
    padded = torch.empty((n, 2 * s + s), dtype=torch.uint8, device="cuda")
    half = objs[:, 2 * s:].clone()
    ov = B.shard_views(objs, k, s)
    pv = B.shard_views(par, m, s)
    rv = [(rebuilt.data_ptr(), rebuilt.stride(0)), (rebuilt.data_ptr() + s, rebuilt.stride(0))]
    sv = [(padded.data_ptr() + s, padded.stride(0)), (padded.data_ptr() + 2 * s, padded.stride(0))]
    hv = [(half.data_ptr(), half.stride(0)), (half.data_ptr() + s, half.stride(0))]
    p01 = [0, 0, 1, 1, 1, 1]
    p23 = [1, 1, 0, 0, 1, 1]
    scratch = objs.clone()  # in-place case writes into a copy
    xv = B.shard_views(scratch, k, s)
    cases = {
        "rec01": (rv + ov[2:] + pv, p01),
        "rec23": (ov[:2] + rv + pv, p23),
        "rec01_half": (rv + hv + pv, p01),
        "rec01_shift": (sv + ov[2:] + pv, p01),
        "rec01_inplace": (xv[:2] + xv[2:] + pv, p01),
    }
    t = {c: [] for c in cases}
    for r in range(rounds + 1):
        order = list(cases) if r % 2 == 0 else list(cases)[::-1]
        for c in order:
            views, present = cases[c]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                B.reconstruct_views(enc, views, present, n, s)
            e1.record()
            torch.cuda.synchronize()
            if r:
                t[c].append(e0.elapsed_time(e1) / reps)
    ok = torch.equal(rebuilt, objs[:, :2 * s]) and torch.equal(padded[:, s:], objs[:, :2 * s])
    ok = ok and torch.equal(scratch, objs)
    for c, v in t.items():
        ms = statistics.median(v)
        print(json.dumps({"case": c, "ms": round(ms, 4), "frac": round(n * 6 * s / ms / 1e6 / 8000, 4),
                          "rebuilt_ok": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
