#!/usr/bin/env python3
"""Probe: can the stripe kernel code host-resident stripes in place, reading
and writing pinned host memory directly over PCIe (no staging ring, no CPU
gather/scatter)?  Compares, on the same pinned ecSplit-layout buffer:

  zerocopy  — a StripePlan over the HOST addresses, launched on the GPU
  ring      — hbec_encode_host / hbec_reconstruct_host (pinned staging ring)

and checks both against the device path.  4+2 @ 1 MiB, n objects.
"""
from __future__ import annotations

import json
import statistics
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402

MiB = 1 << 20
GiB = float(1 << 30)


def main(n=2048, reps=5):
    torch.cuda.set_device(0)
    k, m, S = 4, 2, MiB // 4
    enc = RS.New(k, m)
    dev = torch.empty((n, (k + m) * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(dev, k * S)  # rows: data in [0, k*S), parity after
    views = B.shard_views(dev, k + m, S)
    B.encode_views(enc, views, n, S)
    torch.cuda.synchronize()
    want = dev.cpu()
    host = torch.empty((n, (k + m) * S), dtype=torch.uint8).pin_memory()
    stripes = [(host.data_ptr() + i * host.stride(0), S) for i in range(n)]
    st = torch.cuda.current_stream()

    def reset():
        host.copy_(want)
        host[:, k * S:].zero_()

    res = []

    def emit(name, ts, nbytes, ok):
        med = statistics.median(ts)
        row = {"measure": name, "objects": n, "ms": round(med * 1e3, 3), "object_data_GiB_s": round(n * k * S / med / GiB, 2),
               "pcie_GB_s": round(nbytes / med / 1e9, 2), "ok": ok}
        res.append(row)
        print(json.dumps(row), flush=True)

    # zero-copy encode: plan over host addresses
    plan = B.StripePlan(enc, stripes)
    reset()
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t = time.perf_counter()
        plan.encode(stream=st)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ok = bool(torch.equal(host, want))
    emit("zerocopy_plan_encode", ts[1:], n * (k + m) * S, ok)

    # zero-copy reconstruct {0,1}
    present = [0, 0, 1, 1, 1, 1]
    ts = []
    for _ in range(reps + 1):
        host[:, :2 * S].zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        plan.reconstruct(present, stream=st)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ok = bool(torch.equal(host, want))
    emit("zerocopy_plan_reconstruct01", ts[1:], n * (k + 2) * S, ok)
    del plan

    # staging ring on the same pinned buffer
    reset()
    rows = [r for r in host.numpy()]
    ts = []
    for _ in range(reps + 1):
        t = time.perf_counter()
        enc.EncodeStripes(rows)
        ts.append(time.perf_counter() - t)
    ok = bool(torch.equal(host, want))
    emit("ring_encode_host_pinned", ts[1:], n * (k + m) * S, ok)
    ts = []
    for _ in range(reps + 1):
        host[:, :2 * S].zero_()
        t = time.perf_counter()
        enc.ReconstructStripes(rows, present)
        ts.append(time.perf_counter() - t)
    ok = bool(torch.equal(host, want))
    emit("ring_reconstruct01_host_pinned", ts[1:], n * (k + 2) * S, ok)
    return res


if __name__ == "__main__":
    main()
