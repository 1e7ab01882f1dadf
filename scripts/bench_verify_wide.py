#!/usr/bin/env python3
"""Encoder.Verify of wide policies (k > 8) on the device, any alignment:
gf_verify_wide (one read-only pass) against HBEC_WIDE_VERIFY=0 (round-2
gf_verify_unaligned for k <= 16, scratch recompute above).  n objects of
~1 MiB in ecSplit databufs; % of 8 TB/s on (k+m)*S bytes read.  A clean
batch must verify; one flipped parity byte must flag exactly its object.

    python scripts/bench_verify_wide.py [n_objects]
"""
import json
import os
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402


def t(fn, reps=9):
    fn()
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    torch.cuda.set_device(0)
    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for _ in range(100):
        x.add_(1)
    del x
    for k, m, L in [(10, 4, 1 << 20), (10, 4, 10 * 104864), (12, 4, 1 << 20), (16, 4, 1 << 20), (17, 3, 1 << 20),
                    (20, 4, 1 << 20), (20, 4, 20 * 52432), (32, 8, 1 << 20), (32, 8, 32 * 32767)]:
        s = -(-L // k)
        enc = RS.New(k, m)
        rows = torch.empty((n, (k + m) * s), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(rows, (k + m) * s)
        views = B.shard_views(rows, k + m, s)
        ems = t(lambda: B.encode_views(enc, views, n, s))  # k > 8 at odd offsets: gf_wide apply (HBEC_WIDE_APPLY)
        flags = torch.zeros(n, dtype=torch.int32, device="cuda")
        ms = t(lambda: B.verify_views(enc, views, n, s, flags))
        flags.zero_()
        B.verify_views(enc, views, n, s, flags)
        torch.cuda.synchronize()
        clean = int(flags.count_nonzero().item()) == 0
        rows[n // 3, (k + m) * s - 2] ^= 1
        flags.zero_()
        B.verify_views(enc, views, n, s, flags)
        torch.cuda.synchronize()
        exact = flags.nonzero().flatten().tolist() == [n // 3]
        nb = n * (k + m) * s
        print(json.dumps({"k": k, "m": m, "S": s, "n": n, "wide": os.environ.get("HBEC_WIDE_VERIFY", "1"),
                          "wide_apply": os.environ.get("HBEC_WIDE_APPLY", "1"),
                          "encode_ms": round(ems, 4), "encode_frac": round(nb / (ems * 1e-3) / 8e12, 4),
                          "verify_ms": round(ms, 4), "frac": round(nb / (ms * 1e-3) / 8e12, 4),
                          "clean_ok": clean, "flip_exact": exact}), flush=True)
        del rows, views
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
