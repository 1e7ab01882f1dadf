#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (each its own run) over scripts/odd_sq.py
# for one library; summary per kernel by scripts/pmc_summary.py.
# usage: scripts/pmc_odd.sh TAG SHAPES [LIB]   (N objects: env N, default 2048)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
tag=$1; shapes=$2
[ $# -ge 3 ] && export HBEC_LIB=$ROOT/$3
for c in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $OUT/${tag}_$c
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/${tag}_$c -o run -- python3 $ROOT/scripts/odd_sq.py 3 ${N:-2048} $shapes > $OUT/${tag}_$c.log 2>&1) || exit $?
done
python scripts/pmc_summary.py $OUT/${tag}_FETCH_SIZE $OUT/${tag}_WRITE_SIZE $OUT/${tag}_pmc.json || exit $?
