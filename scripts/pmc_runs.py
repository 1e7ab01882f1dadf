#!/usr/bin/env python3
"""Per-run PMC view: consecutive launches of one kernel in a FETCH_SIZE pass
and a WRITE_SIZE pass of the same script (same launch order) are grouped into
runs; one line per run with median HBM read (2 x FETCH_SIZE, gfx950
correction), write, and kernel-trace duration of the stats pass if given.

    python scripts/pmc_runs.py FETCH_DIR WRITE_DIR [STATS_DIR] [--json OUT]
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys
from pathlib import Path


def short(name: str) -> str:
    m = re.search(r"hbec::(\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def launches(d: Path, counter: str | None):
    rows = []
    for f in sorted(d.glob("*counter_collection.csv" if counter else "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if counter and r["Counter_Name"] != counter:
                continue
            rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]),
                         float(r["Counter_Value"]) if counter else 0.0,
                         int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    return rows


def runs(rows):
    out = []
    for _, k, v, dur in rows:
        if out and out[-1]["kernel"] == k:
            out[-1]["v"].append(v)
            out[-1]["dur"].append(dur)
        else:
            out.append({"kernel": k, "v": [v], "dur": [dur]})
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    jout = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if jout:
        args.remove(jout)
    f = runs(launches(Path(args[0]), "FETCH_SIZE"))
    w = runs(launches(Path(args[1]), "WRITE_SIZE"))
    s = runs(launches(Path(args[2]), None)) if len(args) > 2 else None
    res = []
    for i, (a, b) in enumerate(zip(f, w)):
        if a["kernel"] != b["kernel"]:
            print("run mismatch", i, a["kernel"], b["kernel"], file=sys.stderr)
            break
        if not a["kernel"].startswith(("gf_", "md5", "compare")):
            continue
        row = {"run": i, "kernel": a["kernel"], "launches": len(a["v"]),
               "read_B": 2 * 1024 * statistics.median(a["v"]), "write_B": 1024 * statistics.median(b["v"])}
        if s and i < len(s) and s[i]["kernel"] == a["kernel"]:
            row["ms"] = statistics.median(s[i]["dur"]) / 1e6
        res.append(row)
        print(f"{i:4d} {a['kernel'][:60]:60s} n={len(a['v']):3d} rd={row['read_B']/1e6:10.2f}MB wr={row['write_B']/1e6:10.2f}MB"
              + (f" ms={row['ms']:.4f}" if "ms" in row else ""))
    if jout:
        Path(jout).write_text("\n".join(json.dumps(r) for r in res) + "\n")


if __name__ == "__main__":
    main()
