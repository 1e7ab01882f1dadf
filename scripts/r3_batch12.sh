#!/bin/bash
# Round-3 GPU batch 12: PMC traffic passes (FETCH_SIZE, WRITE_SIZE) and an SQ
# issue pass over bench.py WITH its small / config4 / odd_objects legs, the
# summary written on the box (gpurun_out/r03_pmc.json, also into profiles/ so
# the following bench run reports traffic), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
tag=${1:-r3b12}
B="$ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --config5-objects 0"
mkdir -p $OUT/${tag}_fetch $OUT/${tag}_write $OUT/${tag}_sq
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_fetch -o run -- python3 $B > $OUT/${tag}_fetch.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/${tag}_write -o run -- python3 $B > $OUT/${tag}_write.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/${tag}_sq -o run -- python3 $B > $OUT/${tag}_sq.log 2>&1) || exit $?
timeout -k 10 120 python scripts/pmc_summary.py $OUT/${tag}_fetch $OUT/${tag}_write $OUT/r03_pmc.json > /dev/null || exit $?
cp $OUT/r03_pmc.json profiles/r03_pmc.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $OUT/${tag}_bench.json 2> $OUT/${tag}_bench.err || exit $?
tail -c 600 $OUT/${tag}_bench.json
echo done
