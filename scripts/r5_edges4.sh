#!/bin/bash
# Edge kernel split by object count: GPU suite; kernel traces of one-object
# calls (per-call Verify / encode) and of 16384 short objects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_edges4_tests.log 2>&1 || { tail -40 gpurun_out/r5_edges4_tests.log; exit 1; }
tail -2 gpurun_out/r5_edges4_tests.log
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r5edges4_prof -o run -- python3 $ROOT/scripts/odd_sq.py 30 1 c:8:3:131071:enc,c:4:2:262143:ver > $ROOT/gpurun_out/r5edges4_prof.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r5edges4b_prof -o run -- python3 $ROOT/scripts/odd_sq.py 10 16384 c:8:3:8191:enc > $ROOT/gpurun_out/r5edges4b_prof.log 2>&1) || exit $?
