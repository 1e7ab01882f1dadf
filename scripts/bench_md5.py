#!/usr/bin/env python3
"""ShardHash (GPU MD5) measurements for DESIGN.md — not the headline metric.

For the BASELINE 4+2 @ 1 MiB batch (4096 objects, 6 x 256 KiB shards each)
and 8+3 @ 1 MiB (11 x 128 KiB):
  * md5 of all k+m shards alone (hbec_md5_batch),
  * encode alone, encode then md5 on one stream, and hbec_encode_md5_batch
    (segment pipeline, hash overlapped with the encode),
  * the chain bound: one lane per chain, blocks/chain x VALU per block x 4
    cycles (one wave's issue rate) at the measured clock-free 2.4 GHz,
  * CPU: hashlib MD5 on one core over a bounded sample (GB/s).
Times: HIP events around each call on the current stream, median of reps.
One JSON object per line.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402
from hummingbird_amd import shardhash as H  # noqa: E402

MiB = 1 << 20
VALU_PER_BLOCK = 340  # md5_chains<true,4> main loop: 339 VALU per 64-B block (ISA count)


def timed(fn, reps=7):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def config(k, m, n_obj=4096, obj=MiB):
    S = obj // k
    enc = RS.New(k, m)
    objs = torch.empty((n_obj, k * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * S)
    par = torch.empty((n_obj, m * S), dtype=torch.uint8, device="cuda")
    views = B.shard_views(objs, k, S) + B.shard_views(par, m, S)
    dig = torch.empty((n_obj, k + m, 16), dtype=torch.uint8, device="cuda")
    B.encode_views(enc, views, n_obj, S)
    torch.cuda.synchronize()

    t_md5 = timed(lambda: H.md5_views(views, n_obj, S, digests=dig))
    t_enc = timed(lambda: B.encode_views(enc, views, n_obj, S))

    def seq():
        B.encode_views(enc, views, n_obj, S)
        H.md5_views(views, n_obj, S, digests=dig)

    t_seq = timed(seq)
    t_fused = timed(lambda: H.encode_md5_views(enc, views, n_obj, S, digests=dig))
    torch.cuda.synchronize()
    # spot check against hashlib
    o = n_obj - 1
    host = [objs[o, j * S:(j + 1) * S].cpu().numpy() for j in range(k)] + \
           [par[o, r * S:(r + 1) * S].cpu().numpy() for r in range(m)]
    assert H.hexdigests(dig[o:o + 1])[0] == [hashlib.md5(x.tobytes()).hexdigest() for x in host]
    hashed = n_obj * (k + m) * S
    blocks = S // 64
    bound_ms = blocks * VALU_PER_BLOCK * 4 / 2.4e9 * 1e3
    return {"measure": f"shardhash_{k}+{m}_1MiB", "objects": n_obj, "chains": n_obj * (k + m),
            "chain_bytes": S, "md5_ms": round(t_md5, 3), "md5_GB_s_hashed": round(hashed / t_md5 / 1e6, 1),
            "chain_bound_ms": round(bound_ms, 3), "encode_ms": round(t_enc, 3),
            "encode_then_md5_ms": round(t_seq, 3), "encode_md5_pipelined_ms": round(t_fused, 3),
            "pipelined_vs_sequential": round(t_seq / t_fused, 3)}


def chain_scaling(S=MiB // 4):
    """md5_list launch time vs number of 256 KiB chains: one wave per 64
    chains, so few chains expose one lane's latency per 64-B block."""
    rows = []
    total = 24576
    for spacing in (S, S + 4160):  # power-of-two vs skewed chain starts
        buf = torch.empty((total, spacing), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(buf, spacing)
        for n in (1, 64, 1024, 4096, 24576):
            bufs = [(buf.data_ptr() + i * spacing, S) for i in range(n)]
            dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
            t = timed(lambda: H.md5_list(bufs, digests=dig), reps=5)
            rows.append({"measure": "md5_list_chain_scaling", "chains": n, "chain_bytes": S, "spacing": spacing,
                         "ms": round(t, 3), "us_per_block": round(t * 1e3 / (S // 64), 4),
                         "GB_s_hashed": round(n * S / t / 1e6, 2)})
        del buf
    return rows


def cpu_md5(seconds=3.0):
    buf = np.random.default_rng(0).integers(0, 256, 64 * MiB, dtype=np.uint8).tobytes()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        hashlib.md5(buf).digest()
        n += 1
    t = time.perf_counter() - t0
    return {"measure": "cpu_hashlib_md5_1core", "GB_s": round(n * len(buf) / t / 1e9, 3),
            "cpu": os.uname().machine}


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--label", default="")
    ap.add_argument("--objects", default="4096", help="comma list of batch sizes (objects per call)")
    ap.add_argument("--no-scaling", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    rows = []
    for n in map(int, args.objects.split(",")):
        rows += [config(4, 2, n), config(8, 3, n)]
    rows += ([] if args.no_scaling else chain_scaling()) + ([] if args.no_cpu else [cpu_md5()])
    for r in rows:
        if args.label:
            r["label"] = args.label
            r["segments"] = os.environ.get("HBEC_MD5_SEGMENTS", "8")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
