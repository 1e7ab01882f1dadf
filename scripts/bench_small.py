#!/usr/bin/env python3
"""Small objects at the README bench shape (4 KB objects, /root/reference/
README.md:19-27): 65 536 x 4 KiB, device-resident, 8+3 (S = 512 B) and 4+2
(S = 1 KiB), encode and reconstruct.  Two timings per op:

  stream   - 20 launches back to back on one stream (HIP events, average),
             after 200 settling launches: the clocks dip and recover over the
             first ~10 ms of sustained short launches (profiles/
             r02_small_dvfs_drift.jsonl)
  isolated - one launch after a sync and a 1 GiB write that evicts L2 and the
             256 MiB Infinity Cache of the previous launch's lines (median of 9)

Algorithmic bytes per object: encode (k+m)*S, reconstruct (k+e)*S (SURVEY
§8d).  Outputs are self-checked with Encoder.Verify (a different kernel).
One JSON line per measurement.

    python scripts/bench_small.py [n_objects] [obj_bytes]
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

GiB = float(1 << 30)
PEAK = 8000.0


def emit(name, nbytes, ms, **kw):
    d = {"config": name, "ms": round(ms, 5), "algorithmic_bytes": nbytes,
         "GB_s": round(nbytes / (ms * 1e-3) / 1e9, 1), "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 1e9 / PEAK, 4)}
    d.update(kw)
    print(json.dumps(d), flush=True)


def stream_ms(fn, reps=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def isolated_ms(fn, scrub, reps=9):
    ts = []
    for _ in range(reps):
        scrub.zero_()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def run(k, m, n, size, miss, scrub):
    s = size // k
    enc = RS.New(k, m)
    objs = torch.empty((n, size), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, size)
    par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
    out = torch.empty((n, len(miss) * s), dtype=torch.uint8, device="cuda")
    views = B.shard_views(objs, k, s) + B.shard_views(par, m, s)
    rv = list(views)
    for slot, i in enumerate(miss):
        rv[i] = (out.data_ptr() + slot * s, out.stride(0))
    present = [0 if i in miss else 1 for i in range(k + m)]

    def encode():
        B.encode_views(enc, views, n, s)

    def reconstruct():
        B.reconstruct_views(enc, rv, present, n, s)

    for _ in range(200):  # settle the clocks (see the module docstring)
        encode()
    info = B.kernel_info(k, m, s)
    enc_b, rec_b = n * (k + m) * s, n * (k + len(miss)) * s
    emit(f"{k}+{m} encode {n}x{size} stream", enc_b, stream_ms(encode), kernel=info["kind"],
         tile_bytes=info["tile_bytes"])
    emit(f"{k}+{m} encode {n}x{size} isolated", enc_b, isolated_ms(encode, scrub), kernel=info["kind"])
    emit(f"{k}+{m} reconstruct{set(miss)} {n}x{size} stream", rec_b, stream_ms(reconstruct), kernel=info["kind"])
    emit(f"{k}+{m} reconstruct{set(miss)} {n}x{size} isolated", rec_b, isolated_ms(reconstruct, scrub))
    # self-check: every object's parity verifies (Encoder.Verify, a different
    # kernel, timed too: (k+m)*S read per object); rebuilt shards equal the originals
    flags = torch.zeros(n, dtype=torch.int32, device="cuda")

    def verify():
        B.verify_views(enc, views, n, s, flags)

    emit(f"{k}+{m} verify {n}x{size} stream", enc_b, stream_ms(verify), bound="HBM read")
    emit(f"{k}+{m} verify {n}x{size} isolated", enc_b, isolated_ms(verify, scrub), bound="HBM read")
    torch.cuda.synchronize()
    assert int(flags.count_nonzero()) == 0, "parity does not verify"
    for slot, i in enumerate(miss):
        src = objs[:, i * s:(i + 1) * s] if i < k else par[:, (i - k) * s:(i - k + 1) * s]
        assert torch.equal(out[:, slot * s:(slot + 1) * s], src), miss


def main():
    torch.cuda.set_device(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    scrub = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    run(8, 3, n, size, (0, 1, 2), scrub)
    run(4, 2, n, size, (0, 1), scrub)


if __name__ == "__main__":
    main()
