#!/usr/bin/env python3
"""Turn the two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE, each collected in
its own run with --kernel-trace only) into per-launch HBM bytes per kernel.

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md §HBM):
  * FETCH_SIZE (KiB) reads exactly 1/2 of a wide coalesced streaming read
    -> hbm_read = 2 * FETCH_SIZE * 1024
  * WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores
    -> hbm_write = WRITE_SIZE * 1024

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc.json
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
    return m.group(1) if m else name[:80]


def dispatches(d: Path, counter: str):
    """[(dispatch id, kernel, grid size, counter value, duration)] in dispatch order."""
    out = []
    for f in d.glob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            out.append((int(row["Dispatch_Id"]), short(row["Kernel_Name"]), int(row["Grid_Size"]),
                        float(row["Counter_Value"]), dur))
    return sorted(out)


def per_kernel(rows):
    """{kernel: [(counter value, duration)]} over the launches of the kernel's
    LARGEST grid: a kernel that bench.py also launches for small checks (e.g.
    one-object Verify calls after a plan leg) is reported for its bench-size
    launches, not for the many tiny ones."""
    out = {}
    for _, k, g, c, t in rows:
        out.setdefault(k, []).append((g, c, t))
    res = {}
    for k, v in out.items():
        g = max(x[0] for x in v)
        res[k] = [(c, t) for gg, c, t in v if gg == g]
    return res


def by_leg(rows, legs, mark_blocks):
    """Split the dispatches at bench.py's leg markers (a fill_splitmix launch
    of mark_blocks + i blocks starts leg i); {leg: rows}."""
    out, cur = {}, None
    for r in rows:
        i = r[2] // 256 - mark_blocks
        if r[1] == "fill_splitmix" and r[2] % 256 == 0 and 0 <= i < len(legs):
            cur = legs[i]
            continue
        if cur is not None:
            out.setdefault(cur, []).append(r)
    return out


def summarize(fetch, write):
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("gf_") and not k.startswith("fill") and not k.startswith("md5"):
            continue
        f = [v for v, _ in fetch.get(k, [])]
        w = [v for v, _ in write.get(k, [])]
        rd = 2 * statistics.median(f) * 1024 if f else None
        wr = statistics.median(w) * 1024 if w else None
        kernels[k] = {
            "launches_fetch_pass": len(f), "launches_write_pass": len(w),
            "FETCH_SIZE_KiB_median": statistics.median(f) if f else None,
            "WRITE_SIZE_KiB_median": statistics.median(w) if w else None,
            "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
            "hbm_bytes_per_launch": (rd + wr) if (rd is not None and wr is not None) else None,
        }
    return kernels


def main():
    fetch_dir, write_dir, dst = Path(sys.argv[1]), Path(sys.argv[2]), Path(sys.argv[3])
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench  # the sources the dominant kernel is built from: bench.py trusts only a matching summary

    fr, wr = dispatches(fetch_dir, "FETCH_SIZE"), dispatches(write_dir, "WRITE_SIZE")
    kernels = summarize(per_kernel(fr), per_kernel(wr))
    fl, wl = by_leg(fr, bench.PMC_LEGS, bench.PMC_MARK_BLOCKS), by_leg(wr, bench.PMC_LEGS, bench.PMC_MARK_BLOCKS)
    legs = {leg: summarize(per_kernel(fl.get(leg, [])), per_kernel(wl.get(leg, [])))
            for leg in bench.PMC_LEGS if leg in fl or leg in wl}
    res = {"source": [str(fetch_dir), str(write_dir)],
           "kernel_sources_sha256": bench.kernel_sources_sha256(),
           "odd_sources_sha256": bench.kernel_sources_sha256(bench.ODD_SOURCES),
           "corrections": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count on wide streaming reads); "
                          "write = WRITE_SIZE x 1024",
           "kernels": kernels,
           "legs": legs}
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
