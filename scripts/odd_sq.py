#!/usr/bin/env python3
"""Driver for per-kernel counter passes over the odd-shard kernel families
(VERDICT r03 item 1): each shape is launched `reps` times back to back after
a clock settle, so a rocprofv3 --pmc pass sees runs of one kernel at a time.

    python scripts/odd_sq.py [reps] [n_objects] [shape,...]

Shapes (ecSplit databufs, device-resident, 2048 objects by default):
  a42   aligned 4+2 @ 1 MiB            gf_apply_vec_pipe2<4,2>   (reference point)
  o42   4+2,  S = 262 143              gf_odd<4,2,0>
  v42   4+2 Verify                     gf_odd<4,2,2>
  r42   4+2 reconstruct {0,1}          gf_odd<4,2,0>
  a83   aligned 8+3 @ 1 MiB            gf_apply_vec_pipe<8,3>
  o83   8+3,  S = 131 071              gf_odd<8,3,0>
  r83   8+3 reconstruct {0,1}          gf_odd<8,2,0>
  v83   8+3 Verify                     gf_odd<8,3,2>
  o104  10+4, S = 104 858              gf_odd<10,4,0>
  r104  10+4 reconstruct {0,1}         gf_odd<10,2,0>
  o124  12+4, S = 87 389               gf_odd<12,4,0>
  p124  12+4 object plan, S = 87 392   gf_odd_plan<12,4,...>
  v328  32+8 Verify, S = 32 768 + 3    gf_wide<8,...> verify
One JSON line per shape (median ms, % of 8 TB/s on the algorithmic bytes);
every encode is checked with the product's Verify.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

MiB = 1 << 20
ALL = ["a42", "o42", "a83", "o83", "r83", "v83", "o104", "p124", "v328"]


def main():
    import torch

    from hummingbird_amd import batch as B
    from hummingbird_amd import reedsolomon as RS

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    names = sys.argv[3].split(",") if len(sys.argv) > 3 else ALL
    torch.cuda.set_device(0)

    def timeit(fn):
        fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts)

    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for _ in range(200):
        x.add_(1)
    del x

    def databuf(k, m, s):
        rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(rows, (k + m) * s)
        return rows, B.shard_views(rows, k + m, s)

    def check(enc, views, s):
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.verify_views(enc, views, n, s, flags)
        torch.cuda.synchronize()
        return int(flags.count_nonzero().item()) == 0

    for name in names:
        if name.startswith("w:"):  # w:K:M:S:DI:DO  inputs at i (S + DI), outputs (own array) at r (S + DO)
            _, k, m, s, di, do_ = name.split(":")
            k, m, s, di, do_ = int(k), int(m), int(s), int(di), int(do_)
            op = "skew"
        elif name.startswith("c:"):  # custom: c:K:M:S:OP (OP enc / rec / ver / plan / dplan / dplanp)
            _, k, m, s, op = name.split(":")
            k, m, s = int(k), int(m), int(s)
        else:
          k, m, s, op = {"a42": (4, 2, MiB // 4, "enc"), "o42": (4, 2, 262143, "enc"), "v42": (4, 2, 262143, "ver"), "r42": (4, 2, 262143, "rec"), "a83": (8, 3, MiB // 8, "enc"),
                       "o83": (8, 3, 131071, "enc"), "r83": (8, 3, 131071, "rec"), "v83": (8, 3, 131071, "ver"),
                       "o104": (10, 4, 104858, "enc"), "o124": (12, 4, 87389, "enc"), "r104": (10, 4, 104858, "rec"), "p124": (12, 4, 87392, "plan"), "p42": (4, 2, 262143, "plan"), "p83": (8, 3, 131071, "plan"), "p104": (10, 4, 104858, "plan"),
                       "v328": (32, 8, 32771, "ver"), "v104": (10, 4, 104858, "ver"), "v124": (12, 4, 87389, "ver"),
                       "v32": (3, 2, 349525, "ver"), "o53": (5, 3, 209715, "enc"), "o64": (6, 4, 174763, "enc"), "o102": (10, 2, 104858, "enc"), "o103": (10, 3, 104858, "enc"), "o122": (12, 2, 87389, "enc"), "o123": (12, 3, 87389, "enc"), "v53": (5, 3, 209715, "ver"), "v64": (6, 4, 174763, "ver"), "v102": (10, 2, 104858, "ver"), "v103": (10, 3, 104858, "ver"), "v122": (12, 2, 87389, "ver"), "v123": (12, 3, 87389, "ver"), "p102": (10, 2, 104858, "plan"), "p123": (12, 3, 87389, "plan"), "p64": (6, 4, 174763, "plan"), "v84": (8, 4, 131071, "ver"), "v93": (9, 3, 116509, "ver"), "v73": (7, 3, 149797, "ver"), "v62": (6, 2, 174763, "ver"), "v82": (8, 2, 131071, "ver"), "v63": (6, 3, 174763, "ver"), "o63": (6, 3, 174763, "enc"), "o73": (7, 3, 149797, "enc"), "o62": (6, 2, 174763, "enc"), "o82": (8, 2, 131071, "enc"), "o84": (8, 4, 131071, "enc"), "o93": (9, 3, 116509, "enc"), "p63": (6, 3, 174763, "plan"), "p73": (7, 3, 149797, "plan"), "p42b": (4, 2, 262141, "plan"), "c42": (4, 2, 262143, "cplan"), "c83": (8, 3, 131071, "cplan"), "c104": (10, 4, 104858, "cplan"),
                       # random sizes (the nursery batch shape): object plans of n objects, S uniform in
                       # [4 KiB / k, 1 MiB / k], odd
                       "x42": (4, 2, 0, "rplan"), "x83": (8, 3, 0, "rplan"), "x104": (10, 4, 0, "rplan"), "x124": (12, 4, 0, "rplan")}[name]
        enc = RS.New(k, m)
        row = {"lib": os.environ.get("HBEC_LIB", "default"), "label": os.environ.get("AB_LABEL", ""), "round": int(os.environ.get("AB_ROUND", "0")),
               "shape": name, "k": k, "m": m, "S": s, "n": n, "op": op}
        if op == "rplan":
            rng = __import__("numpy").random.default_rng(0x48424543 + k * 100 + m)
            sizes = [int(x) | 1 for x in rng.integers(4096 // k, (1 << 20) // k + 1, n)]
            row["S"] = "random"
        if op in ("cplan", "rplan"):
            if op == "cplan":
                sizes = [s if i % 2 else max(17, s // 256 + 7) for i in range(n)]
            # object plan of two size classes, alternating: ~4 KiB and ~1 MiB objects, odd S
            d = torch.empty(sum(k * x for x in sizes), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(d.view(1, -1), d.numel())
            par = torch.empty(sum(m * x for x in sizes), dtype=torch.uint8, device="cuda")
            objs, do, po = [], 0, 0
            for x in sizes:
                objs.append((d.data_ptr() + do, par.data_ptr() + po, x))
                do += k * x
                po += m * x
            plan = B.StripePlan(enc, objects=objs)
            ms = timeit(plan.encode)
            nb = sum((k + m) * x for x in sizes)
            plan.encode()
            flags = torch.zeros(1, dtype=torch.int32, device="cuda")
            ok = True
            for (a_, b_, x) in objs[:64]:
                views = [(a_ + j * x, 0) for j in range(k)] + [(b_ + r * x, 0) for r in range(m)]
                flags.zero_()
                B.verify_views(enc, views, 1, x, flags)
                ok = ok and int(flags.item()) == 0
            torch.cuda.synchronize()
            row["ok"] = ok
            del plan, d, par
        elif op == "skew":
            din = torch.empty((n, k * (s + di) + 256), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(din, din.shape[1])
            dout = torch.empty((n, m * (s + do_) + 256), dtype=torch.uint8, device="cuda")
            views = [(din.data_ptr() + i * (s + di), din.stride(0)) for i in range(k)] + \
                    [(dout.data_ptr() + r * (s + do_), dout.stride(0)) for r in range(m)]
            B.encode_views(enc, views, n, s)
            ms = timeit(lambda: B.encode_views(enc, views, n, s))
            nb = n * (k + m) * s
            row["ok"] = check(enc, views, s)
            row["DI"], row["DO"] = di, do_
            del din, dout, views
        elif op in ("dplan", "dplanp"):
            # the databuf layout of "enc" (shard i at row + i S) coded through an object plan;
            # dplanp: objects listed in the order 0, n/2, 1, n/2 + 1, ... (concurrent waves
            # on rows half the batch apart)
            rows, views = databuf(k, m, s)
            order = list(range(n)) if op == "dplan" else [i // 2 + (n // 2) * (i % 2) for i in range(n)]
            plan = B.StripePlan(enc, objects=[(rows.data_ptr() + i * rows.stride(0),
                                               rows.data_ptr() + i * rows.stride(0) + k * s, s) for i in order])
            ms = timeit(plan.encode)
            nb = n * (k + m) * s
            row["ok"] = check(enc, views, s)
            del plan, rows, views
        elif op == "plan":
            d = torch.empty((n, k * s), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(d, k * s)
            par = torch.empty((n, m * s), dtype=torch.uint8, device="cuda")
            plan = B.StripePlan(enc, objects=[(d.data_ptr() + i * d.stride(0), par.data_ptr() + i * par.stride(0), s)
                                              for i in range(n)])
            ms = timeit(plan.encode)
            nb = n * (k + m) * s
            row["ok"] = check(enc, B.shard_views(d, k, s) + B.shard_views(par, m, s), s)
            del plan, d, par
        else:
            rows, views = databuf(k, m, s)
            B.encode_views(enc, views, n, s)
            if op == "enc":
                ms = timeit(lambda: B.encode_views(enc, views, n, s))
                nb = n * (k + m) * s
            elif op == "rec":
                present = [0, 0] + [1] * (k + m - 2)
                ms = timeit(lambda: B.reconstruct_views(enc, views, present, n, s))
                nb = n * (k + 2) * s
            else:
                flags = torch.zeros(n, dtype=torch.int32, device="cuda")
                ms = timeit(lambda: B.verify_views(enc, views, n, s, flags))
                nb = n * (k + m) * s
            row["ok"] = check(enc, views, s)
            del rows, views
        row["ms"] = round(ms, 4)
        row["frac"] = round(nb / (ms * 1e-3) / 8e12, 4)
        print(json.dumps(row), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
