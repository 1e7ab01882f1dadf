#!/usr/bin/env python3
"""A/B kernel variants of libhbec in ONE process, interleaved rounds.

    python scripts/tune.py build            # on the CPU container: compile variants
    python scripts/tune.py run [--rounds R] # on the GPU: time + cross-check

Each variant = extra -D definitions (kernel shape) and/or env (grid sizing),
built into tune_build/<name>/libhbec.so.  The run loads every variant with
ctypes, runs the 4+2 @ 1 MiB x 4096 workload (encode + reconstruct{0,1}),
checks every variant's parity and rebuilt bytes against the first variant's,
and prints per-variant median / min kernel time and achieved GB/s.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUTDIR = ROOT / "tune_build"

# Build-time variants override a tuning.h constant (-D); runtime variants set
# a tune_knob environment variable, which only a tuning build reads, so every
# variant is built with HBEC_TUNE=1.  The product values are in tuning.h.
VARIANTS = {
    "cur": ([], {}),
    # packed kernel (short shards, e.g. 8+3 of 4 KiB objects)
    "pk_vec": ([], {"HBEC_PACKED": "0"}),
    "pk_u2": (["HBEC_PACKED_U_BIG=2"], {}),
    "pk_sb1": (["HBEC_PACKED_BLOCKS_SMALL=1"], {}),
    "pk_sb3": (["HBEC_PACKED_BLOCKS_SMALL=3"], {}),
    "pk_max2k": ([], {"HBEC_PACKED_MAX_SHARD": "2048"}),
    # packed verify (short shards): run scripts/bench_small.py with HBEC_LIB=tune_build/<name>/libhbec.so
    "vp_u1": (["HBEC_VERIFY_PACKED_U_SMALL=1"], {}),
    "vp_u4": (["HBEC_VERIFY_PACKED_U_SMALL=4"], {}),
    "vp_b1": (["HBEC_VERIFY_PACKED_BLOCKS_SMALL=1", "HBEC_VERIFY_PACKED_BLOCKS_BIG=1"], {}),
    "md5d4": (["HBEC_MD5_DEPTH=4"], {}),
    "ch256k": ([], {"HBEC_CHUNK_TILES": str(256 << 10)}),
    "ch4m": ([], {"HBEC_CHUNK_TILES": str(4 << 20)}),
    "sleep4": (["HBEC_PIPE2_SLEEP=4"], {}),
    "sleep12": (["HBEC_PIPE2_SLEEP=12"], {}),
    "u2big": (["HBEC_PIPE_U_BIG=2"], {}),
    "b2": ([], {"HBEC_BLOCKS_PER_CU": "2"}),
}


def build(names):

    from hummingbird_amd import build as hb

    for n in names:
        defs, _ = VARIANTS[n]
        d = OUTDIR / n
        hb.build(defs=["HBEC_TUNE=1"] + list(defs), lib=d / "libhbec.so", objdir=d / "obj", verbose=False)
        print("built", n, flush=True)


_HOLD = []  # buffers of earlier runs (--allocs): kept so the next run's land elsewhere


def run(names, rounds, n_obj, launches, k=4, m=2, size=1 << 20):
    import torch

    from hummingbird_amd import _native as N

    torch.cuda.set_device(0)
    s = size // k
    e = min(m, 3)  # erased data shards 0..e-1
    libs = {}
    for n in names:
        _, env = VARIANTS[n]
        old = {var: os.environ.get(var) for var in env}
        os.environ.update(env)
        h = C.CDLL(str(OUTDIR / n / "libhbec.so"))
        for var, v in old.items():
            if v is None:
                os.environ.pop(var, None)
            else:
                os.environ[var] = v
        for name, res, args in N._SIG:
            if not hasattr(h, name):  # a variant built before a newer entry point
                continue
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
        codec = C.c_void_p()
        assert h.hbec_new(k, m, C.byref(codec)) == 0
        libs[n] = (h, codec)

    objs = torch.empty((n_obj, k * s), dtype=torch.uint8, device="cuda")
    _HOLD.append(objs)
    h0 = libs[names[0]][0]
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert h0.hbec_fill_splitmix(C.c_void_p(objs.data_ptr()), n_obj, k * s, k * s, 0x48424543, 0, stream) == 0
    shared_p = torch.zeros((n_obj, m * s), dtype=torch.uint8, device="cuda")
    shared_r = torch.zeros((n_obj, e * s), dtype=torch.uint8, device="cuda")
    _HOLD.extend([shared_p, shared_r])
    parity = {n: shared_p for n in names}
    rebuilt = {n: shared_r for n in names}
    ok = {n: [True, True] for n in names}
    ref_p = None

    def views(n):
        enc = [(objs.data_ptr() + j * s, k * s) for j in range(k)] + \
              [(parity[n].data_ptr() + r * s, m * s) for r in range(m)]
        rec = list(enc)
        for i in range(e):
            rec[i] = (rebuilt[n].data_ptr() + i * s, e * s)
        mk = lambda vs: (N.View * (k + m))(*[N.View(b, st) for b, st in vs])  # noqa: E731
        return mk(enc), mk(rec)

    vv = {n: views(n) for n in names}
    present = (C.c_uint8 * (k + m))(*([0] * e + [1] * (k + m - e)))
    times = {n: {"enc": [], "rec": []} for n in names}
    for rnd in range(rounds):
        for n in names:
            h, codec = libs[n]
            ve, vr = vv[n]
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * launches + 1)]
            torch.cuda.synchronize()
            evs[0].record()
            for i in range(launches):
                assert h.hbec_encode_batch(codec, ve, n_obj, s, stream) == 0
                evs[2 * i + 1].record()
                assert h.hbec_reconstruct_batch(codec, vr, present, n_obj, s, 0, stream) == 0
                evs[2 * i + 2].record()
            torch.cuda.synchronize()
            if ref_p is None:
                ref_p = shared_p.clone()
            if rnd == rounds - 1:
                ok[n] = [bool(torch.equal(shared_p, ref_p)), bool(torch.equal(shared_r, objs[:, :e * s]))]
                shared_p.zero_()
                shared_r.zero_()
            if rnd > 0:  # round 0 = warmup
                for i in range(launches):
                    times[n]["enc"].append(evs[2 * i].elapsed_time(evs[2 * i + 1]))
                    times[n]["rec"].append(evs[2 * i + 1].elapsed_time(evs[2 * i + 2]))
    bytes_per_launch = n_obj * (k + m) * s
    rec_bytes = n_obj * (k + e) * s
    res = []
    for n in names:
        okp, okr = ok[n]
        h = libs[n][0]
        tb, st, bpc = C.c_int(), C.c_int(), C.c_int()
        h.hbec_kernel_info(k, m, s, C.byref(tb), C.byref(st), C.byref(bpc))
        e_ms = statistics.median(times[n]["enc"])
        r = statistics.median(times[n]["rec"])
        row = {"variant": n, "k": k, "m": m, "enc_ms_med": round(e_ms, 4), "rec_ms_med": round(r, 4),
               "enc_ms_min": round(min(times[n]["enc"]), 4), "rec_ms_min": round(min(times[n]["rec"]), 4),
               "enc_GBs": round(bytes_per_launch / e_ms / 1e6, 1), "rec_GBs": round(rec_bytes / r / 1e6, 1),
               "frac": round((bytes_per_launch + rec_bytes) / (e_ms + r) / 1e6 / 8000, 4), "parity_ok": okp, "rebuilt_ok": okr,
               "tile": tb.value, "blocks_per_cu": bpc.value}
        res.append(row)
        print(json.dumps(row), flush=True)
    return res


def run_layout(reps=8):
    """Encode/reconstruct time vs. buffer placement (default lib)."""
    import torch

    from hummingbird_amd import _native as N
    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS

    torch.cuda.set_device(0)
    n_obj, S = 4096, 1 << 18
    enc = RS.New(4, 2)
    pool_bytes = (4 * S + 64 * 1024) * n_obj + 2 * (2 * S + 64 * 1024) * n_obj + (64 << 20)
    pool = torch.empty(pool_bytes, dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    present = [0, 0, 1, 1, 1, 1]
    results = []
    for obj_pad in (0, 4096, 16384, 65536):
        for par_off in (0, 4096, 1 << 20, (32 << 20) + 4096):
            ostride = 4 * S + obj_pad
            pstride = 2 * S + obj_pad
            obase = base
            pbase = base + ostride * n_obj + par_off
            pbase = (pbase + 4095) // 4096 * 4096 + (par_off % 4096)
            rbase = pbase + pstride * n_obj + 4096
            # every byte any kernel touches must lie inside the pool
            assert obase + ostride * n_obj <= base + pool_bytes
            assert rbase + pstride * (n_obj - 1) + 2 * S <= base + pool_bytes, "layout exceeds pool"
            assert pbase + pstride * (n_obj - 1) + 2 * S <= rbase
            assert N.lib().hbec_fill_splitmix(C.c_void_p(obase), n_obj, 4 * S, ostride, 0x48424543, 0,
                                               C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
            ev = [(obase + j * S, ostride) for j in range(4)] + [(pbase + r * S, pstride) for r in range(2)]
            rv = [(rbase, pstride), (rbase + S, pstride)] + ev[2:]
            te, tr = [], []
            for r in range(reps + 1):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                B.encode_views(enc, ev, n_obj, S)
                e1.record()
                B.reconstruct_views(enc, rv, present, n_obj, S)
                e2.record()
                torch.cuda.synchronize()
                if r:
                    te.append(e0.elapsed_time(e1))
                    tr.append(e1.elapsed_time(e2))
            e, rr = statistics.median(te), statistics.median(tr)
            row = {"obj_pad": obj_pad, "par_off": par_off, "enc_ms": round(e, 4), "rec_ms": round(rr, 4),
                   "frac": round(2 * n_obj * 6 * S / (e + rr) / 1e6 / 8000, 4)}
            results.append(row)
            print(json.dumps(row), flush=True)
    return results


def run_copy_sweep(reps=8):
    import torch

    torch.cuda.set_device(0)
    h = C.CDLL(str(OUTDIR / "probe.so"))
    h.probe_copy_variant.restype = C.c_int
    h.probe_copy_variant.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_int,
                                     C.c_void_p]
    n = 2 << 30
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    src.random_(0, 255)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    best = []
    for block in (256, 512, 1024):
        for u in (1, 2, 4, 8):
            for nt in (0, 1):
                for grid in (256, 512, 1024, 2048, 4096, 16384):
                    ts = []
                    for r in range(reps + 1):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        rc = h.probe_copy_variant(u, nt, src.data_ptr(), dst.data_ptr(), n, grid, block, st)
                        assert rc == 0, rc
                        e1.record()
                        torch.cuda.synchronize()
                        if r:
                            ts.append(e0.elapsed_time(e1))
                    med = statistics.median(ts)
                    row = {"block": block, "u": u, "nt": nt, "grid": grid, "ms": round(med, 4),
                           "GBs": round(2 * n / med / 1e6, 1)}
                    best.append(row)
                    print(json.dumps(row), flush=True)
    assert torch.equal(src, dst)
    best.sort(key=lambda r: -r["GBs"])
    print("TOP", json.dumps(best[:8]))


def run_xor_sweep(reps=8):
    import torch

    torch.cuda.set_device(0)
    h = C.CDLL(str(OUTDIR / "probe.so"))
    h.probe_xor_variant.restype = C.c_int
    h.probe_xor_variant.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p]
    n_obj, S = 4096, 1 << 18
    objs = torch.empty((n_obj, 4 * S), dtype=torch.uint8, device="cuda")
    out = torch.empty((n_obj, 2 * S), dtype=torch.uint8, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows = []
    for u in (0, 1, 4):  # 0 = shard-interleaved layout
        for grid in (256, 512, 1024, 2048, 4096):
            ts = []
            for r in range(reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert h.probe_xor_variant(u, objs.data_ptr(), out.data_ptr(), n_obj, S, grid, st) == 0
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            row = {"u": u, "grid": grid, "ms": round(med, 4), "GBs": round(n_obj * 6 * S / med / 1e6, 1)}
            rows.append(row)
            print(json.dumps(row), flush=True)


def run_seq(reps=6):
    """Encode-only and reconstruct-only back-to-back sequences (default lib)."""
    import torch

    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS

    torch.cuda.set_device(0)
    n, S = 4096, 1 << 18
    enc = RS.New(4, 2)
    objs = torch.empty((n, 4 * S), dtype=torch.uint8, device="cuda")
    par = torch.empty((n, 2 * S), dtype=torch.uint8, device="cuda")
    reb = torch.empty((n, 2 * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, 4 * S)
    ev = B.shard_views(objs, 4, S) + B.shard_views(par, 2, S)
    rv = B.shard_views(reb, 2, S) + ev[2:]
    pres = [0, 0, 1, 1, 1, 1]
    # reconstruct of the PARITY shards only (inputs = 4 data shards, like encode, other decode rows)
    rv_p = ev[:4] + B.shard_views(reb, 2, S)
    seqs = {
        "enc": lambda: B.encode_views(enc, ev, n, S),
        "rec01": lambda: B.reconstruct_views(enc, rv, pres, n, S),
        "rec45": lambda: B.reconstruct_views(enc, rv_p, [1, 1, 1, 1, 0, 0], n, S),
    }
    for rnd in range(3):
        for name, fn in seqs.items():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
            torch.cuda.synchronize()
            evs[0].record()
            for i in range(reps):
                fn()
                evs[i + 1].record()
            torch.cuda.synchronize()
            ts = [evs[i].elapsed_time(evs[i + 1]) for i in range(reps)]
            print(json.dumps({"seq": name, "round": rnd, "ms": [round(t, 4) for t in ts],
                              "med": round(statistics.median(ts[1:]), 4)}), flush=True)
    torch.cuda.synchronize()
    assert torch.equal(reb, par)  # rec45 regenerates the parity


def build_probe():
    import subprocess
    OUTDIR.mkdir(exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-x", "hip", str(ROOT / "scripts" / "hbm_probe.hip"), "-o", str(OUTDIR / "probe.so")],
                   check=True)
    print("built probe")


def run_probe(reps=10):
    import torch

    torch.cuda.set_device(0)
    h = C.CDLL(str(OUTDIR / "probe.so"))
    h.probe_launch.restype = C.c_int
    h.probe_launch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                               C.c_int, C.c_void_p]
    n_obj, S = 4096, 1 << 18
    objs = torch.randint(0, 255, (n_obj, 4 * S), dtype=torch.uint8, device="cuda")
    out = torch.empty((n_obj, 2 * S), dtype=torch.uint8, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    cases = []
    for grid in (1024, 2048, 4096, 8192):
        cases += [("read4G", 0, objs, out, 4 << 30, 4 << 30, 0, grid),
                  ("write2G", 1, objs, out, 2 << 30, 2 << 30, 0, grid),
                  ("copy2G", 2, objs, out, 2 << 30, 4 << 30, 0, grid),
                  ("xor42_objmajor", 3, objs, out, 0, 6 << 30, 0, grid),
                  ("xor42_offmajor", 3, objs, out, 0, 6 << 30, 1, grid),
                  ("xor40_read", 4, objs, out, 0, 4 << 30, 0, grid)]
    for name, which, a, b, n, traffic, mode, grid in cases:
        ts = []
        for r in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert h.probe_launch(which, a.data_ptr(), b.data_ptr(), n, n_obj, S, mode, grid, st) == 0
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        med = statistics.median(ts)
        print(json.dumps({"probe": name, "grid": grid, "ms": round(med, 4),
                          "GBs": round(traffic / med / 1e6, 1), "frac": round(traffic / med / 1e6 / 8000, 4)}),
              flush=True)
    h.probe_write_variant.restype = C.c_int
    h.probe_write_variant.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
    names = ["flat_plain", "flat_nt", "flat_plain_u4", "flat_nt_u4", "buf_aux0", "buf_nt", "buf_sc1", "buf_sc0sc1",
             "buf_ntsc1", "buf_sc0", "flat_nt_u8"]
    for grid in (512, 1024, 2048, 4096):
        for v, nm in enumerate(names):
            ts = []
            for r in range(reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert h.probe_write_variant(v, out.data_ptr(), 2 << 30, grid, st) == 0
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(json.dumps({"probe": "w_" + nm, "grid": grid, "ms": round(med, 4),
                              "GBs": round((2 << 30) / med / 1e6, 1), "frac": round((2 << 30) / med / 1e6 / 8000, 4)}),
                  flush=True)
    # torch / runtime references
    for name, fn, traffic in [("torch_copy2G", lambda: out.view(-1).copy_(objs.view(-1)[: 2 << 30]), 4 << 30)]:
        ts = []
        for r in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        med = statistics.median(ts)
        print(json.dumps({"probe": name, "ms": round(med, 4), "GBs": round(traffic / med / 1e6, 1),
                          "frac": round(traffic / med / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "probe", "build_probe", "layout", "copysweep", "xorsweep", "seq"])
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--objects", type=int, default=4096)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--size", type=int, default=1 << 20, help="object bytes (shard = size / k)")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--allocs", type=int, default=1,
                    help="repeat the run on this many fresh buffer sets (earlier ones stay allocated, "
                         "so each set lands on different physical memory)")
    a = ap.parse_args()
    names = a.variants.split(",")
    if a.cmd == "build":
        build(names)
    elif a.cmd == "build_probe":
        build_probe()
    elif a.cmd == "probe":
        run_probe()
    elif a.cmd == "seq":
        run_seq()
    elif a.cmd == "xorsweep":
        run_xor_sweep()
    elif a.cmd == "copysweep":
        run_copy_sweep()
    elif a.cmd == "layout":
        run_layout()
    else:
        for i in range(a.allocs):
            if a.allocs > 1:
                print(json.dumps({"alloc_set": i}), flush=True)
            run(names, a.rounds, a.objects, a.launches, a.k, a.m, a.size)
