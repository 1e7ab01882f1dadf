"""Child process of tests/test_gpu_rings.py (run as a script, not collected).

More concurrent host-path callers than host rings: T threads on a library
started with HBEC_HOST_RINGS set low (the parent sets 2) each run
hbec_encode_host, hbec_encode_host_md5 and hbec_reconstruct_host over their
own stripes, pageable and pinned (hbec_host_alloc), of three shard lengths
(1 MiB objects, an odd 1 MiB - 3 B object, 4 KiB).  Every result is compared
with the CPU oracle (oracle/gf_oracle.c parity, hashlib MD5, the original
data for a rebuild).  Round 2's soak stalled with callers making rings on
demand (DESIGN.md §5 "Concurrency soak"); the bound must queue callers
without losing a wake-up.  Prints one JSON line; exit status 0 = all good.

    HBEC_HOST_RINGS=2 python tests/ring_stress.py THREADS ITERS
"""
from __future__ import annotations

import hashlib
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from hummingbird_amd import reedsolomon as RS  # noqa: E402
from oracle import coracle as CO  # noqa: E402

K, M = 4, 2
N = K + M
SIZES = [1 << 20, (1 << 20) - 3, 4096]  # object bytes; S = ceil(len / k)


def make_stripes(enc, tid, pinned, bufs):
    out = []
    rng = np.random.default_rng(0x5249 + tid)
    for j, size in enumerate(SIZES):
        s = -(-size // K)
        if pinned:
            hb = RS.HostBuffer(N * s)
            bufs.append(hb)
            st = hb.array[:N * s]
        else:
            st = np.empty(N * s, dtype=np.uint8)
        st[:K * s] = rng.integers(0, 256, K * s, dtype=np.uint8)
        st[K * s:] = 0
        want, _ = CO.encode_batch(K, M, st[:K * s].reshape(1, K * s).copy())
        out.append((st, s, st.copy(), want[0]))
        out[-1][2][K * s:] = want[0]
    return out


def worker(enc, tid, iters, pinned, errors, counts, bufs):
    try:
        stripes = make_stripes(enc, tid, pinned, bufs)
        for it in range(iters):
            op = (tid + it) % 3
            sts = [st for st, _, _, _ in stripes]
            for st, s, _, _ in stripes:
                st[K * s:] = 0x11
            if op == 0:
                enc.EncodeStripes(sts)
            elif op == 1:
                digs = enc.EncodeStripesMD5(sts)
                for (st, s, full, _), d in zip(stripes, digs):
                    want = [hashlib.md5(full[i * s:(i + 1) * s].tobytes()).hexdigest() for i in range(N)]
                    if d != want:
                        raise AssertionError(f"thread {tid} iter {it}: MD5 differs (S = {s})")
            else:
                enc.EncodeStripes(sts)
                for st, s, _, _ in stripes:
                    st[0:s] = 0x77
                    st[4 * s:5 * s] = 0x77
                enc.ReconstructStripes(sts, [0, 1, 1, 1, 0, 1])
            for st, s, full, want in stripes:
                if not np.array_equal(st[K * s:], want):
                    raise AssertionError(f"thread {tid} iter {it} op {op}: parity differs from the oracle (S = {s})")
                if not np.array_equal(st, full):
                    raise AssertionError(f"thread {tid} iter {it} op {op}: stripe differs (S = {s})")
            counts[tid] += 1
    except Exception as e:  # noqa: BLE001 — reported to the parent
        errors.append(f"{type(e).__name__}: {e}")


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    enc = RS.New(K, M)
    errors, counts, bufs = [], [0] * threads, []
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(enc, t, iters, t % 2 == 0, errors, counts, bufs))
           for t in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    for b in bufs:
        b.free()
    print(json.dumps({"threads": threads, "iters": iters, "calls": sum(counts), "seconds": round(dt, 2),
                      "errors": errors[:5]}), flush=True)
    return 0 if not errors and sum(counts) == threads * iters else 1


if __name__ == "__main__":
    sys.exit(main())
