#!/usr/bin/env python3
"""Host-path (PCIe-inclusive) rates for DESIGN.md — not the headline metric.

The reference path starts and ends in host memory (nursery file / HTTP body
in, shard PUT bodies out: objectserver/ecobj.go:689-811, ecutils.go:26-72).
Two measurements:

 1. pipelined batch: objects in pinned host memory -> H2D (k*S per object) ->
    encode kernel -> D2H (m*S per object), chunked and double-buffered on three
    HIP streams (copy-in / compute / copy-out), for 4+2 @ 1 MiB; same for a
    reconstruct{0,1} (survivors in, 2 rebuilt shards out).
 2. per-call Encoder.Encode through the C ABI on pageable host buffers (what a
    drop-in ecSplit call does per stripe), 1 MiB objects, sequential.

Prints one JSON object per measurement.
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402
from scripts import _common as U  # noqa: E402

MiB = 1 << 20
GiB = float(1 << 30)


def pipelined(op: str, n_obj=4096, chunk=256, reps=3):
    k, m, S = 4, 2, MiB // 4
    enc = RS.New(k, m)
    n_in = 4 if op == "encode" else 4  # survivors read per object
    n_out = 2
    host_in = torch.empty((n_obj, n_in * S), dtype=torch.uint8).pin_memory()
    host_out = torch.empty((n_obj, n_out * S), dtype=torch.uint8).pin_memory()
    dev_objs = torch.empty((n_obj, k * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(dev_objs, k * S)
    dev_par = torch.empty((n_obj, m * S), dtype=torch.uint8, device="cuda")
    B.encode_objects(enc, dev_objs, dev_par, S)
    torch.cuda.synchronize()
    if op == "encode":
        host_in.copy_(dev_objs.cpu())
        want = dev_par.cpu()
    else:  # survivors 2,3,P0,P1 -> rebuild 0,1
        host_in.copy_(torch.cat([dev_objs[:, 2 * S:], dev_par], dim=1).cpu())
        want = dev_objs[:, :2 * S].cpu()
    del dev_objs, dev_par
    d_in = [torch.empty((chunk, n_in * S), dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_out = [torch.empty((chunk, n_out * S), dtype=torch.uint8, device="cuda") for _ in range(2)]
    s_in, s_cmp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    present = [0, 0, 1, 1, 1, 1]

    def run():
        done_out = [None, None]
        for c in range(n_obj // chunk):
            b = c % 2
            lo, hi = c * chunk, (c + 1) * chunk
            with torch.cuda.stream(s_in):
                if done_out[b] is not None:
                    s_in.wait_event(done_out[b])  # buffer b's previous D2H has finished
                d_in[b].copy_(host_in[lo:hi], non_blocking=True)
                e_in = torch.cuda.Event()
                e_in.record(s_in)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(e_in)
                if op == "encode":
                    views = B.shard_views(d_in[b], 4, S) + B.shard_views(d_out[b], 2, S)
                    B.encode_views(enc, views, chunk, S, stream=s_cmp)
                else:
                    views = B.shard_views(d_out[b], 2, S) + B.shard_views(d_in[b], 4, S)
                    B.reconstruct_views(enc, views, present, chunk, S, stream=s_cmp)
                e_cmp = torch.cuda.Event()
                e_cmp.record(s_cmp)
            with torch.cuda.stream(s_out):
                s_out.wait_event(e_cmp)
                host_out[lo:hi].copy_(d_out[b], non_blocking=True)
                e_out = torch.cuda.Event()
                e_out.record(s_out)
                done_out[b] = e_out
        torch.cuda.synchronize()

    run()
    assert torch.equal(host_out, want), "host-path output differs"
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    obj_bytes = n_obj * k * S
    return {"measure": f"host_path_pipelined_{op}", "objects": n_obj, "chunk_objects": chunk,
            "seconds": round(t, 4),
            "object_data_GiB_s": round(obj_bytes / t / GiB, 2),
            "algorithmic_GiB_s": round(n_obj * (n_in + n_out) * S / t / GiB, 2),
            "pcie_GB_s_h2d_plus_d2h": round(n_obj * (n_in + n_out) * S / t / 1e9, 2),
            "objects_per_s": round(n_obj / t, 1)}


def library_host_path(op: str, n_obj=4096, reps=3, mem="pageable", k=4, m=2, obj=MiB):
    """hbec_encode_host / hbec_reconstruct_host.  mem="pageable": numpy stripes
    through the library's pinned ring (CPU gather -> H2D -> kernel -> D2H ->
    scatter).  mem="pinned": stripes in hbec_host_alloc memory, coded in place
    by the GPU over PCIe (zero-copy, no CPU copies)."""
    S = obj // k
    enc = RS.New(k, m)
    hb = None
    if mem == "pinned":
        hb = RS.HostBuffer(n_obj * (k + m) * S)
        pool = hb.array.reshape(n_obj, (k + m) * S)
    else:
        pool = np.empty((n_obj, (k + m) * S), dtype=np.uint8)
    pool[:, :k * S] = U.objects_host(n_obj, k * S)
    stripes = [pool[i] for i in range(n_obj)]
    # the stripe descriptor array is built once, outside the timed calls: the
    # library's rate, not Python's per-stripe ctypes marshalling (~1 us/stripe)
    import ctypes as C

    from hummingbird_amd import _native as N
    arr = enc._stripes(stripes)
    present = (C.c_uint8 * (k + m))(*([0, 0] + [1] * (k + m - 2)))
    L = N.lib()
    run = (lambda: RS.check(L.hbec_encode_host(enc.handle, arr, n_obj))) if op == "encode" else \
        (lambda: RS.check(L.hbec_reconstruct_host(enc.handle, arr, n_obj, present, 0)))
    RS.check(L.hbec_encode_host(enc.handle, arr, n_obj))  # warm up the ring
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    if op == "encode":
        assert U.verify_stripe(enc, pool[7].copy())
    res = {"measure": f"library_host_path_{op}_{mem}", "k": k, "m": m, "object_bytes": obj, "objects": n_obj,
           "seconds": round(t, 4),
           "object_data_GiB_s": round(n_obj * k * S / t / GiB, 2),
           "algorithmic_GiB_s": round(n_obj * (k + m) * S / t / GiB, 2),
           "pcie_GB_s": round(n_obj * (k + m) * S / t / 1e9, 2), "objects_per_s": round(n_obj / t, 1)}
    del stripes, pool
    if hb is not None:
        hb.free()
    return res


def batched_callers(n_threads=64, per_thread=32, mem="pageable"):
    """Many concurrent callers, one 1 MiB object each per call, through the
    batching driver (what concurrent Stabilize goroutines would do).
    mem="pinned": the callers' stripes are hbec_host_alloc buffers (zero-copy)."""
    import threading

    k, m, S = 4, 2, MiB // 4
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=96 << 20, max_wait_us=300)
    n = n_threads * per_thread
    hb = None
    if mem == "pinned":
        hb = RS.HostBuffer(n * (k + m) * S)
        pool = hb.array.reshape(n, (k + m) * S)
    else:
        pool = np.empty((n, (k + m) * S), dtype=np.uint8)
    pool[:, :k * S] = U.objects_host(n, k * S)

    def worker(t):
        for i in range(t * per_thread, (t + 1) * per_thread):
            bat.Encode(pool[i])

    bat.Encode(pool[0])  # warm the ring
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    t = time.perf_counter() - t0
    st = bat.stats()
    bat.close()
    assert U.verify_stripe(enc, pool[n - 1].copy())
    del pool
    if hb is not None:
        hb.free()
    return {"measure": f"batcher_concurrent_Encode_1MiB_{mem}", "threads": n_threads, "objects": n,
            "seconds": round(t, 4), "object_data_GiB_s": round(n * k * S / t / GiB, 2),
            "us_per_object": round(t / n * 1e6, 1), "batches": st["batches"]}


def library_host_path_md5(n_obj=4096, reps=3, mem="pageable", k=4, m=2):
    """hbec_encode_host_md5: the library host path plus the ShardHash of all
    k+m shards of every stripe, hashed on the GPU per chunk."""
    S = MiB // k
    enc = RS.New(k, m)
    hb = None
    if mem == "pinned":
        hb = RS.HostBuffer(n_obj * (k + m) * S)
        pool = hb.array.reshape(n_obj, (k + m) * S)
    else:
        pool = np.empty((n_obj, (k + m) * S), dtype=np.uint8)
    import hashlib
    pool[:, :k * S] = U.objects_host(n_obj, k * S)
    stripes = [pool[i] for i in range(n_obj)]
    hs = enc.EncodeStripesMD5(stripes)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        hs = enc.EncodeStripesMD5(stripes)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    assert hs[9] == [hashlib.md5(pool[9, i * S:(i + 1) * S]).hexdigest() for i in range(k + m)]
    res = {"measure": f"library_host_path_encode_md5_{mem}", "k": k, "m": m, "objects": n_obj,
           "seconds": round(t, 4), "object_data_GiB_s": round(n_obj * k * S / t / GiB, 2),
           "hashed_GiB_s": round(n_obj * (k + m) * S / t / GiB, 2), "objects_per_s": round(n_obj / t, 1)}
    del stripes, pool
    if hb is not None:
        hb.free()
    return res


def small_objects_host():
    """The README's 4 KB shape through the host path: 262 144 x 4 KiB stripes
    (1 GiB of objects) per call, 4+2 (S = 1 KiB) and 8+3 (S = 512 B)."""
    out = []
    for k, m in ((4, 2), (8, 3)):
        for mem in ("pageable", "pinned"):
            out.append(library_host_path("encode", n_obj=262144, mem=mem, k=k, m=m, obj=4096))
    return out


def md5_vs_encode():
    """Encode + ShardHash against Encode alone, same stripes, 4+2 and 8+3 @
    1 MiB, pageable and pinned: the cost of the hash next to the encode."""
    out = []
    for k, m in ((4, 2), (8, 3)):
        for mem in ("pageable", "pinned"):
            e = library_host_path("encode", mem=mem, k=k, m=m)
            h = library_host_path_md5(mem=mem, k=k, m=m)
            out.append({"measure": f"host_path_encode_md5_vs_encode_{k}+{m}_{mem}", "objects": 4096,
                        "encode_s": e["seconds"], "encode_md5_s": h["seconds"],
                        "ratio": round(h["seconds"] / e["seconds"], 3)})
    return out


def batched_callers_md5(n_threads=64, per_thread=32):
    import threading

    k, m, S = 4, 2, MiB // 4
    enc = RS.New(k, m)
    bat = RS.Batcher(enc, max_batch_bytes=96 << 20, max_wait_us=300)
    n = n_threads * per_thread
    pool = np.empty((n, (k + m) * S), dtype=np.uint8)
    pool[:, :k * S] = U.objects_host(n, k * S)
    out = [None] * n

    def worker(t):
        for i in range(t * per_thread, (t + 1) * per_thread):
            out[i] = bat.EncodeMD5(pool[i])

    bat.EncodeMD5(pool[0])
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    t = time.perf_counter() - t0
    st = bat.stats()
    bat.close()
    import hashlib
    assert out[n - 1] == [hashlib.md5(pool[n - 1, i * S:(i + 1) * S]).hexdigest() for i in range(k + m)]
    return {"measure": "batcher_concurrent_EncodeMD5_1MiB", "threads": n_threads, "objects": n,
            "seconds": round(t, 4), "object_data_GiB_s": round(n * k * S / t / GiB, 2),
            "us_per_object": round(t / n * 1e6, 1), "batches": st["batches"]}


def auditor_pass(n_files=4096, size=MiB // 4):
    """hbec_md5_host over host 'shard files' (one GPU lane per file) vs one
    CPU core of hashlib."""
    import hashlib

    from hummingbird_amd import shardhash as H
    rng = np.random.default_rng(1)
    files = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(n_files)]
    H.md5_host(files[:8])
    t0 = time.perf_counter()
    got = H.md5_host(files)
    t = time.perf_counter() - t0
    t1 = time.perf_counter()
    want = [hashlib.md5(f).hexdigest() for f in files[:256]]
    tc = (time.perf_counter() - t1) * n_files / 256
    assert got[:256] == want
    return {"measure": "auditor_md5_host", "files": n_files, "file_bytes": size, "seconds": round(t, 4),
            "GiB_s": round(n_files * size / t / GiB, 2), "cpu_1core_GiB_s": round(n_files * size / tc / GiB, 2)}


def per_call(n_calls=200, mem="pageable"):
    """One klauspost Encode per 1 MiB object, sequential (the naive drop-in).
    mem="pinned": the shards live in hbec_host_alloc memory (zero-copy)."""
    k, m, S = 4, 2, MiB // 4
    enc = RS.New(k, m)
    rng = np.random.default_rng(0)
    obj = rng.integers(0, 256, k * S, dtype=np.uint8)
    hb = None
    if mem == "pinned":
        hb = RS.HostBuffer((k + m) * S)
        shards = [hb.array[i * S:(i + 1) * S] for i in range(k + m)]
        for j in range(k):
            shards[j][:] = obj[j * S:(j + 1) * S]
    else:
        shards = [obj[j * S:(j + 1) * S].copy() for j in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
    enc.Encode(shards)
    t0 = time.perf_counter()
    for _ in range(n_calls):
        enc.Encode(shards)
    t = time.perf_counter() - t0
    assert U.verify_shards(enc, shards)
    del shards
    if hb is not None:
        hb.free()
    return {"measure": f"per_call_Encode_{mem}_1MiB", "calls": n_calls, "us_per_call": round(t / n_calls * 1e6, 1),
            "object_data_GiB_s": round(n_calls * k * S / t / GiB, 3)}


def main():
    torch.cuda.set_device(0)
    steps = [lambda: pipelined("encode"), lambda: pipelined("reconstruct"),
             lambda: library_host_path("encode"), lambda: library_host_path("reconstruct"),
             lambda: library_host_path("encode", mem="pinned"), lambda: library_host_path("reconstruct", mem="pinned"),
             library_host_path_md5, batched_callers, lambda: batched_callers(mem="pinned"), batched_callers_md5,
             auditor_pass, per_call, lambda: per_call(mem="pinned"), md5_vs_encode, small_objects_host]
    only = sys.argv[1:]
    for i, f in enumerate(steps):
        if only and str(i) not in only:
            continue
        r = f()
        for x in (r if isinstance(r, list) else [r]):
            print(json.dumps(x), flush=True)


if __name__ == "__main__":
    main()
