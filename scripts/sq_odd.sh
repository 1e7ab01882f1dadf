#!/bin/bash
# SQ issue counters + kernel-trace stats over scripts/odd_sq.py for one library.
# usage: scripts/sq_odd.sh TAG SHAPES [LIB]   (N objects: env N, default 2048)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
tag=$1; shapes=$2
[ $# -ge 3 ] && export HBEC_LIB=$ROOT/$3
mkdir -p $OUT/${tag}_sq1 $OUT/${tag}_prof
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/${tag}_sq1 -o run -- python3 $ROOT/scripts/odd_sq.py 3 ${N:-2048} $shapes > $OUT/${tag}_sq1.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_prof -o run -- python3 $ROOT/scripts/odd_sq.py 10 ${N:-2048} $shapes > $OUT/${tag}_prof.log 2>&1) || exit $?
python scripts/sq_summary.py $OUT/${tag}_sq1.json $OUT/${tag}_sq1 --only gf_ || exit $?
echo done
