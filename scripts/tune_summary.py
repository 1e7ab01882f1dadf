#!/usr/bin/env python3
"""Median per (shape, variant) of scripts/tune_odd.py JSON lines.

    python scripts/tune_summary.py FILE.jsonl
"""
import collections
import json
import statistics
import sys

agg = collections.defaultdict(list)
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    r = json.loads(line)
    agg[(r["k"], r["m"], r.get("S") or 0, r["layout"], r["variant"])].append(r)
for key in sorted(agg):
    rows = agg[key]
    out = []
    for op in ("encode", "reconstruct", "verify"):
        v = [x[op] for x in rows if x.get(op)]
        if v:
            out.append(f"{op[:3]} {statistics.median(v):.3f}")
    print(key, " ".join(out), all(x.get("ok", True) for x in rows))
