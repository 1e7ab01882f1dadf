#!/usr/bin/env python3
"""Why does 4+2 reconstruct{0,1} trail encode by 2-4 %?  Same kernel, same
4-in / 2-out byte counts; only where the streams live differs.  Cases (all
through hbec_apply_batch with fixed non-zero coefficients, so only the
addresses change), timed interleaved:

  enc          in obj[0..3]            out par[0,1]        (encode)
  rec01        in obj[2,3] par[0,1]    out reb[0,1]        (bench.py's reconstruct)
  rec01_pfirst in par[0,1] obj[2,3]    out reb[0,1]        (input order swapped)
  rec01_inpl   in obj[2,3] par[0,1]    out obj[0,1]        (rebuilt in place)
  rec23        in obj[0,1] par[0,1]    out reb[0,1]
  rec01_pad    rec01 with the rebuilt array's rows padded by 64 KiB
  rec01_ppad   rec01 with the parity array's rows padded by 64 KiB

Prints one JSON line per case (ms, % of 8 TB/s) per repetition of the sweep.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import batch as B  # noqa: E402
from scripts.bench_configs import interleaved  # noqa: E402

MiB = 1 << 20
N, S = 4096, 256 << 10
COEF = [[208, 107, 104, 210], [107, 208, 210, 104]]


def rows(t, idx, pitch=None):
    row = pitch if pitch is not None else t.stride(0)
    return [(t.data_ptr() + i * S, row) for i in idx]


def main(reps=3):
    torch.cuda.set_device(0)
    obj = torch.empty((N, 4 * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(obj, 4 * S)
    par = torch.empty((N, 2 * S), dtype=torch.uint8, device="cuda")
    reb = torch.empty((N, 2 * S), dtype=torch.uint8, device="cuda")
    reb_pad = torch.empty((N, 2 * S + (64 << 10)), dtype=torch.uint8, device="cuda")
    par_pad = torch.empty((N, 2 * S + (64 << 10)), dtype=torch.uint8, device="cuda")
    scratch = torch.empty_like(obj)  # in-place target copy, so obj's inputs stay intact

    def ap(ins, outs):
        return lambda: B.apply_views(2, 4, COEF, ins, outs, N, S)

    scratch.copy_(obj)
    cases = {
        "enc": ap(rows(obj, [0, 1, 2, 3]), rows(par, [0, 1])),
        "rec01": ap(rows(obj, [2, 3]) + rows(par, [0, 1]), rows(reb, [0, 1])),
        "rec01_pfirst": ap(rows(par, [0, 1]) + rows(obj, [2, 3]), rows(reb, [0, 1])),
        "rec01_inpl": ap(rows(scratch, [2, 3]) + rows(par, [0, 1]), rows(scratch, [0, 1])),
        "rec23": ap(rows(obj, [0, 1]) + rows(par, [0, 1]), rows(reb, [0, 1])),
        "rec01_pad": ap(rows(obj, [2, 3]) + rows(par, [0, 1]), rows(reb_pad, [0, 1])),
        "rec01_ppad": ap(rows(obj, [2, 3]) + rows(par_pad, [0, 1]), rows(reb, [0, 1])),
    }
    nbytes = N * 6 * S
    for rep in range(reps):
        t = interleaved(cases)
        for c, ms in t.items():
            print(json.dumps({"rep": rep, "case": c, "ms": round(ms, 4),
                              "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)


def pitch_sweep(pads=(0, 4096, 16384, 65536, 131072, 262144, 524288), obj_pads=(0, 65536), insts=1):
    """Encode and reconstruct{0,1} vs the parity / rebuilt rows' pitch
    (2 S + pad) and the object rows' pitch (4 S + obj_pad), interleaved.
    With insts > 1 every (obj_pad, par_pad) pair gets that many separate
    allocations, so physical placement luck shows as spread."""
    torch.cuda.set_device(0)
    cases, keep = {}, []
    for inst, op in [(i, o) for i in range(insts) for o in obj_pads]:
        obj = torch.empty((N, 4 * S + op), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(obj, 4 * S)
        keep.append(obj)
        for pp in pads:
            par = torch.empty((N, 2 * S + pp), dtype=torch.uint8, device="cuda")
            reb = torch.empty((N, 2 * S + pp), dtype=torch.uint8, device="cuda")
            keep += [par, reb]
            cases[(inst, op, pp, "enc")] = (lambda o=obj, p=par: B.apply_views(2, 4, COEF, rows(o, [0, 1, 2, 3]),
                                                                       rows(p, [0, 1]), N, S))
            cases[(inst, op, pp, "rec01")] = (lambda o=obj, p=par, r=reb: B.apply_views(
                2, 4, COEF, rows(o, [2, 3]) + rows(p, [0, 1]), rows(r, [0, 1]), N, S))
    nbytes = N * 6 * S
    for rep in range(2):
        t = interleaved(cases, rounds=4)
        for (inst, op, pp, c), ms in t.items():
            print(json.dumps({"sweep": "pitch", "rep": rep, "inst": inst, "obj_pad": op, "par_pad": pp, "case": c,
                              "ms": round(ms, 4), "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)


def alloc_sweep(insts=3):
    """Encode and reconstruct{0,1} over buffers from torch's allocator, plain
    hipMalloc and hipExtMallocWithFlags(hipDeviceMallocContiguous), `insts`
    separate allocations each: is the allocation-to-allocation spread
    physical placement (page fragments / channels), and does contiguous
    memory remove it?"""
    import ctypes as C
    from hummingbird_amd import _native as Nat
    torch.cuda.set_device(0)
    hip = C.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    keep, cases = [], {}

    def raw(nbytes, contiguous):
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), nbytes, 4) if contiguous else hip.hipMalloc(C.byref(p), nbytes)
        if rc != 0:
            raise RuntimeError(f"allocation failed: {rc}")
        return p.value

    for inst in range(insts):
        for kind in ("torch", "hipMalloc", "contiguous"):
            if kind == "torch":
                ts = [torch.empty((N, w * S), dtype=torch.uint8, device="cuda") for w in (4, 2, 2)]
                keep.append(ts)
                o, p_, r = (t.data_ptr() for t in ts)
            else:
                o, p_, r = (raw(N * w * S, kind == "contiguous") for w in (4, 2, 2))
            Nat.lib().hbec_fill_splitmix(C.c_void_p(o), N, 4 * S, 4 * S, B.HBEC_SEED, 0, C.c_void_p(0))
            ov = lambda idx, base=o: [(base + i * S, 4 * S) for i in idx]  # noqa: E731
            pv = lambda idx, base=p_: [(base + i * S, 2 * S) for i in idx]  # noqa: E731
            rv = lambda idx, base=r: [(base + i * S, 2 * S) for i in idx]  # noqa: E731
            cases[(kind, inst, "enc")] = (lambda a=ov([0, 1, 2, 3]), b=pv([0, 1]):
                                          B.apply_views(2, 4, COEF, a, b, N, S))
            cases[(kind, inst, "rec01")] = (lambda a=ov([2, 3]) + pv([0, 1]), b=rv([0, 1]):
                                            B.apply_views(2, 4, COEF, a, b, N, S))
    torch.cuda.synchronize()
    nbytes = N * 6 * S
    for rep in range(2):
        t = interleaved(cases, rounds=4)
        for (kind, inst, c), ms in t.items():
            print(json.dumps({"sweep": "alloc", "rep": rep, "alloc": kind, "inst": inst, "case": c,
                              "ms": round(ms, 4), "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)


def contig_sweep():
    """Pitch / offset sweep inside ONE physically contiguous arena
    (hipDeviceMallocContiguous), where virtual offsets are physical offsets,
    so the HBM channel hash sees exactly the layout chosen here.  Each layout:
    objects at 0 with pitch 4S + opad, parity at obj_end + gap with pitch
    2S + ppad, rebuilt right after parity (same pitch); encode and
    reconstruct{0,1} timed interleaved per layout; the baseline layout is
    repeated at the start, middle and end to expose drift."""
    import ctypes as C
    from hummingbird_amd import _native as Nat
    torch.cuda.set_device(0)
    hip = C.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    cap = N * (8 * S) + N * (3 * 262144) + (64 << 20)
    p = C.c_void_p()
    if hip.hipExtMallocWithFlags(C.byref(p), cap, 4) != 0:
        raise RuntimeError("contiguous arena allocation failed")
    arena = p.value
    base = [(0, 0, 0)]
    layouts = base + [(op, pp, 0) for op in (0, 4096, 16384, 65536) for pp in (0, 4096, 16384, 65536)
                      if (op, pp) != (0, 0)][:8] + base + \
        [(op, pp, 0) for op in (0, 4096, 16384, 65536) for pp in (0, 4096, 16384, 65536) if (op, pp) != (0, 0)][8:] + \
        [(0, 0, g) for g in (4096, 1 << 20, 2 << 20, 8 << 20)] + base
    nbytes = N * 6 * S
    for li, (op, pp, gap) in enumerate(layouts):
        opitch, ppitch = 4 * S + op, 2 * S + pp
        o = arena
        pb = o + N * opitch + gap
        r = pb + N * ppitch
        assert r + N * ppitch <= arena + cap
        Nat.lib().hbec_fill_splitmix(C.c_void_p(o), N, 4 * S, opitch, B.HBEC_SEED, 0, C.c_void_p(0))
        ov = [(o + i * S, opitch) for i in range(4)]
        pv = [(pb + i * S, ppitch) for i in range(2)]
        rv = [(r + i * S, ppitch) for i in range(2)]
        cases = {"enc": lambda: B.apply_views(2, 4, COEF, ov, pv, N, S),
                 "rec01": lambda: B.apply_views(2, 4, COEF, ov[2:] + pv, rv, N, S)}
        t = interleaved(cases, rounds=6)
        for c, ms in t.items():
            print(json.dumps({"sweep": "contig", "layout": li, "obj_pad": op, "par_pad": pp, "gap": gap, "case": c,
                              "ms": round(ms, 4), "frac_of_8TBs": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["contig"]:
        contig_sweep()
        sys.exit(0)
    if sys.argv[1:] == ["alloc"]:
        alloc_sweep()
        sys.exit(0)
    if sys.argv[1:] == ["pitch"]:
        pitch_sweep()
    elif sys.argv[1:] == ["pitch2"]:
        pitch_sweep(pads=(0, 4096, 8192, 12288, 16384, 24576, 32768, 49152), obj_pads=(0, 16384), insts=2)
    else:
        main()
