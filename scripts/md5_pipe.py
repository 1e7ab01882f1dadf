#!/usr/bin/env python3
"""Device-resident Encode + ShardHash of 4096 x 1 MiB 4+2 objects
(hbec_encode_md5_batch) next to MD5 alone and Encode alone, one JSON line;
the pipeline's environment knobs are echoed in `label` (scripts/md5_pipe_sweep.sh).

    python scripts/md5_pipe.py [k m]
"""
import hashlib
import json
import os
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from hummingbird_amd import batch as B  # noqa: E402
from hummingbird_amd import reedsolomon as RS  # noqa: E402
from hummingbird_amd import shardhash as H  # noqa: E402


def timed(fn, reps=15):
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
    k, m = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4, 2)
    n, S = 4096, (1 << 20) // k
    torch.cuda.set_device(0)
    enc = RS.New(k, m)
    objs = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(objs, k * S)
    par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    views = B.shard_views(objs, k, S) + B.shard_views(par, m, S)
    dig = torch.empty((n, k + m, 16), dtype=torch.uint8, device="cuda")
    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for _ in range(100):
        x.add_(1)
    del x
    row = {"k": k, "m": m, "objects": n,
           "label": ",".join(f"{v}={os.environ[v]}" for v in sorted(os.environ) if v.startswith("HBEC_MD5") or v == "HBEC_LIB"),
           "round": int(os.environ.get("AB_ROUND", "0"))}
    row["fused_ms"] = round(timed(lambda: H.encode_md5_views(enc, views, n, S, digests=dig)), 4)
    row["md5_ms"] = round(timed(lambda: H.md5_views(views, n, S, digests=dig)), 4)
    row["encode_ms"] = round(timed(lambda: B.encode_views(enc, views, n, S)), 4)
    row["fused_ms_2"] = round(timed(lambda: H.encode_md5_views(enc, views, n, S, digests=dig)), 4)
    torch.cuda.synchronize()
    for o in (0, n - 1):
        host = [objs[o, j * S:(j + 1) * S].cpu().numpy() for j in range(k)] + \
               [par[o, r * S:(r + 1) * S].cpu().numpy() for r in range(m)]
        assert H.hexdigests(dig[o:o + 1])[0] == [hashlib.md5(h.tobytes()).hexdigest() for h in host]
    row["digests_ok"] = True
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
