#!/bin/bash
# Round-3 GPU batch 9 (final kernels): bench line, rocprofv3 kernel stats of the
# same command, the two PMC traffic passes, one SQ issue pass, and the layout probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
tag=${1:-r3b9}
B="$ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --no-small --config5-objects 0"
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $OUT/${tag}_bench.json 2> $OUT/${tag}_bench.err || exit $?
tail -c 400 $OUT/${tag}_bench.json
mkdir -p $OUT/${tag}_prof $OUT/${tag}_fetch $OUT/${tag}_write $OUT/${tag}_sq
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_prof -o run -- python3 $ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-path --no-small --config5-objects 0 > $OUT/${tag}_prof.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_fetch -o run -- python3 $B > $OUT/${tag}_fetch.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_write -o run -- python3 $B > $OUT/${tag}_write.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/${tag}_sq -o run -- python3 $B > $OUT/${tag}_sq.log 2>&1) || exit $?
timeout -k 10 200 ./scripts/layout_probe.bin > $OUT/${tag}_layout_probe.jsonl 2>&1 || exit $?
echo done
