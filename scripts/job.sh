#!/bin/bash
# One GPU job: optional GPU tests, an interleaved library A/B over
# scripts/odd_sq.py shapes, optional kernel trace.  It replaces the
# per-experiment batch files of rounds 4-5 (their job lists are kept in
# profiles/README.md, "Retired job scripts").
# usage: scripts/job.sh OUT.jsonl SHAPES LIB[:VAR=VAL[:VAR=VAL]] ...
#   env TESTS="tests/test_x.py ..."  run these -m gpu tests first (stop on failure)
#       AB_N=n                      objects per shape (default 2048)
#       TRACE=shapes                rocprof kernel trace of odd_sq over these shapes after the A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
out=$1; shapes=$2; shift 2
tag=$(basename "$out" .jsonl)
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$shapes" ] && [ $# -gt 0 ]; then
  timeout -k 10 1000 bash scripts/ab_odd.sh "gpurun_out/$out" "$shapes" "$@" || exit $?
fi
if [ -n "${TRACE:-}" ]; then
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${tag}_prof -o run \
    -- python3 $ROOT/scripts/odd_sq.py 10 ${AB_N:-2048} $TRACE > $ROOT/gpurun_out/${tag}_prof.log 2>&1) || exit $?
fi
echo job-done
