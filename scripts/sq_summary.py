#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc SQ_* passes per kernel: counters summed over the
kernel's dispatches (all of one name), the register / LDS footprint the trace
records, and the derived fractions of wave cycles (SQ_WAVE_CYCLES,
SQ_WAIT_*, SQ_ACTIVE_INST_* all count quad-cycles on gfx950,
MI355X_MICROARCH.md):
  frac_wait_any       parked on s_waitcnt / barrier (memory latency)
  frac_wait_inst_any  ready but not issued (issue stall)
  frac_active_valu    cycles issuing VALU
  valu_per_wave_cycle = SQ_INSTS_VALU * 4 / (SQ_WAVE_CYCLES * 4) per wave

    python scripts/sq_summary.py OUT.json DIR [DIR ...] [--only PREFIX,...]
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    m = re.search(r"hbec::(\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    args = [a for a in sys.argv[1:]]
    only = None
    if "--only" in args:
        i = args.index("--only")
        only = args[i + 1].split(",")
        del args[i:i + 2]
    out, dirs = Path(args[0]), [Path(a) for a in args[1:]]
    sums: dict = defaultdict(lambda: defaultdict(float))
    meta: dict = {}
    disp: dict = defaultdict(set)
    for d in dirs:
        for f in sorted(d.rglob("*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if only and not k.startswith(tuple(only)):
                    continue
                sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((str(f), r["Dispatch_Id"], r["Counter_Name"]))
                meta[k] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r.get("Accum_VGPR_Count") or 0),
                           "sgpr": int(r["SGPR_Count"]), "lds": int(r["LDS_Block_Size"]),
                           "scratch": int(r["Scratch_Size"]), "grid": int(r["Grid_Size"]),
                           "wg": int(r["Workgroup_Size"])}
    res = {}
    for k, c in sums.items():
        row = dict(meta[k])
        names = {n for _, _, n in disp[k]}
        row["dispatches_per_counter"] = len(disp[k]) // max(1, len(names))
        row.update({n: v for n, v in sorted(c.items())})
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n, key in (("SQ_WAIT_ANY", "frac_wait_any"), ("SQ_WAIT_INST_ANY", "frac_wait_inst_any"),
                           ("SQ_ACTIVE_INST_VALU", "frac_active_valu"), ("SQ_ACTIVE_INST_ANY", "frac_active_any"),
                           ("SQ_ACTIVE_INST_VMEM", "frac_active_vmem"), ("SQ_ACTIVE_INST_SCA", "frac_active_sca")):
                if n in c:
                    row[key] = round(c[n] / wc, 4)
        if "SQ_BUSY_CYCLES" in c and "SQ_WAVE_CYCLES" in c and c["SQ_BUSY_CYCLES"]:
            # mean resident waves per SQ while busy (SQ_BUSY_CYCLES counts per SE-SQ cycles)
            row["wave_cycles_per_busy_cycle"] = round(c["SQ_WAVE_CYCLES"] / c["SQ_BUSY_CYCLES"], 2)
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c and c["SQ_WAVES"]:
            row["valu_insts_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"])
        res[k] = row
    out.write_text(json.dumps({"source": [str(d) for d in dirs], "kernels": res}, indent=1) + "\n")
    for k, r in sorted(res.items()):
        print(f"{k[:58]:58s} v={r['vgpr']:3d}+{r['agpr']:3d} wait={r.get('frac_wait_any', '-')} "
              f"stall={r.get('frac_wait_inst_any', '-')} valu={r.get('frac_active_valu', '-')}")


if __name__ == "__main__":
    main()
