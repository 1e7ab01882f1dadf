#!/usr/bin/env python3
"""Host path (PCIe-inclusive) for pinned ecSplit databufs of arbitrary object
sizes: n objects of 1 MiB - (1..15) B (S % 16 != 0, stripes at odd offsets)
next to n objects of exactly 1 MiB, 4+2 and 8+3, through EncodeStripes
(hbec_encode_host).  Run once with HBEC_ZC_UNALIGNED=0 (odd stripes staged
through the ring, the round-1 path) and once without (zero-copy through the
unaligned kernel).  One JSON line per shape; outputs self-checked with the
product's Verify (scripts/_common.py: no oracle here).

    python scripts/bench_host_odd.py [label] [n_objects] [md5]

With "md5", also Encode + ShardHash (hbec_encode_host_md5) of the same
stripes: path taken, cost over Encode alone, sample digests vs hashlib.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import reedsolomon as RS  # noqa: E402
from scripts import _common as U  # noqa: E402

GiB = float(1 << 30)


def run(label, k, m, n, odd, md5=False):
    rng = np.random.default_rng(k * 10 + m)
    layout, off = [], 0
    for _ in range(n):
        size = (1 << 20) - (int(rng.integers(1, 16)) if odd else 0)
        s = -(-size // k)
        layout.append((off, s, size))
        off += (k + m) * s
    hb = RS.HostBuffer(off + 64)
    a = hb.array
    src = U.objects_host(1, 1 << 20)[0]
    for o, s, size in layout:
        a[o:o + size] = src[:size]
        a[o + size:o + k * s] = 0
    stripes = [a[o:o + (k + m) * s] for o, s, _ in layout]
    enc = RS.New(k, m)
    enc.EncodeStripes(stripes)  # warm-up (rings, records)
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        enc.EncodeStripes(stripes)
        ts.append(time.perf_counter() - t)
    t = statistics.median(ts)
    ok = all(U.verify_stripe(enc, stripes[i]) for i in (0, n // 2, n - 1))
    data = sum(size for _, _, size in layout)
    row = {"label": label, "k": k, "m": m, "objects": n, "sizes": "1 MiB - (1..15) B" if odd else "1 MiB",
           "zc_unaligned": os.environ.get("HBEC_ZC_UNALIGNED", "1"), "ms": round(t * 1e3, 2),
           "object_data_GiB_s": round(data / t / GiB, 2), "verify_ok": ok}
    if md5:
        # Encode + ShardHash of every shard (hbec_encode_host_md5) on the same
        # stripes: which path it took (hbec_host_md5_stats) and its cost over
        # Encode alone; digests of a sample against hashlib
        import ctypes as C
        import hashlib

        from hummingbird_amd import _native as N

        def stats():
            zc, ring = C.c_uint64(), C.c_uint64()
            N.lib().hbec_host_md5_stats(C.byref(zc), C.byref(ring))
            return zc.value, ring.value

        enc.EncodeStripesMD5(stripes)
        z0, r0 = stats()
        th = []
        for _ in range(5):
            t1 = time.perf_counter()
            hs = enc.EncodeStripesMD5(stripes)
            th.append(time.perf_counter() - t1)
        z1, r1 = stats()
        tm = statistics.median(th)
        good = all(hs[i] == [hashlib.md5(stripes[i][j * layout[i][1]:(j + 1) * layout[i][1]]).hexdigest()
                             for j in range(k + m)] for i in (0, 1, n // 2, n - 1))
        row.update({"md5_ms": round(tm * 1e3, 2), "md5_over_encode": round(tm / t, 3),
                    "md5_path": {"zero_copy_calls": z1 - z0, "ring_calls": r1 - r0}, "digests_ok": good})
    print(json.dumps(row), flush=True)
    del stripes
    hb.free()


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    md5 = "md5" in sys.argv[3:]
    for k, m in [(4, 2), (8, 3)]:
        for odd in (False, True):
            run(label, k, m, n, odd, md5)


if __name__ == "__main__":
    main()
