#!/usr/bin/env python3
"""Per-dispatch summary of one kernel from a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats averages every dispatch of the process, the warm-up ones
included; the GPU ramps its clocks over the first ~10 launches after start
(1.5 -> 1.08 ms for the headline kernel, profiles/r02_ramp_kernel_trace.txt).
bench.py's roofline is timed over the measured steps only, so this prints the
average over the dispatches after the first `--skip` (bench.py's 2 x warmup)
to compare like with like.

    python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv \
        --kernel gf_apply_vec_pipe2 --skip 20 --out profiles/r02_kernel_trace_summary.json
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True, help="substring of Kernel_Name")
    ap.add_argument("--skip", type=int, default=0, help="leading dispatches to drop (warm-up)")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    timed = dur[a.skip:]
    if not timed:
        raise SystemExit(f"no dispatches of {a.kernel!r} after skipping {a.skip}")
    out = {
        "kernel": rows[0]["Kernel_Name"],
        "dispatches": len(dur),
        "skipped_warmup": a.skip,
        "all_avg_ns": statistics.mean(dur),
        "timed_avg_ns": statistics.mean(timed),
        "timed_median_ns": statistics.median(timed),
        "timed_min_ns": min(timed),
        "timed_max_ns": max(timed),
        # bench.py alternates Encode, Reconstruct
        "timed_even_avg_ns": statistics.mean(timed[0::2]),
        "timed_odd_avg_ns": statistics.mean(timed[1::2]) if len(timed) > 1 else None,
        "warmup_ns": dur[:a.skip],
    }
    text = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
