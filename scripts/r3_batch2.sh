#!/bin/bash
# Round-3 GPU batch 2: bench line, then rocprofv3 kernel stats and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE, each in its own run) over the odd-shape
# benches (scripts/bench_odd.py: strided odd shapes + stripe plans;
# scripts/bench_objplan_wide.py: k > 8 object plans).  Each step has its own
# time limit; the first failure ends the batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
tag=${1:-r3b2}
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > "$OUT/${tag}_bench.json" 2> "$OUT/${tag}_bench.err" || exit $?
tail -1 "$OUT/${tag}_bench.json"
for s in bench_odd bench_objplan_wide; do
  mkdir -p "$OUT/${tag}_${s}_stats" "$OUT/${tag}_${s}_fetch" "$OUT/${tag}_${s}_write"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${tag}_${s}_stats" -o run -- python3 "$ROOT/scripts/$s.py" > "$OUT/${tag}_${s}_stats.log" 2>&1) || exit $?
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/${tag}_${s}_fetch" -o run -- python3 "$ROOT/scripts/$s.py" > "$OUT/${tag}_${s}_fetch.log" 2>&1) || exit $?
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/${tag}_${s}_write" -o run -- python3 "$ROOT/scripts/$s.py" > "$OUT/${tag}_${s}_write.log" 2>&1) || exit $?
  echo "$s profiled"
done
(cd /tmp && timeout -k 10 60 rocprofv3 -L > "$OUT/${tag}_counters.txt" 2>&1) || true
echo done
