#!/bin/bash
# Round-3 GPU batch 23: rocprofv3 --kernel-trace --stats over the default bench
# line on the final round-3 tree (headline + small / config4 / odd_objects
# legs), and the headline kernel's per-dispatch summary over the timed steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT/r3b23_prof; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r3b23_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 10 --no-cpu-baseline > $OUT/r3b23_bench.json 2> $OUT/r3b23_bench.err) || exit $?
ls $OUT/r3b23_prof
tr=$(find $OUT/r3b23_prof -name '*kernel_trace.csv' | head -n 1)
timeout -k 10 120 python scripts/trace_summary.py "$tr" --kernel gf_apply_vec_pipe2 --skip 20 --out $OUT/r3b23_trace_summary.json || exit $?
echo done
