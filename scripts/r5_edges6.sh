#!/bin/bash
# Plan edge kernel with 64 + 64 slots when every stripe is longer than 160 B:
# GPU suite, and a kernel trace of the random-size object plans.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_edges6_tests.log 2>&1 || { tail -40 gpurun_out/r5_edges6_tests.log; exit 1; }
tail -2 gpurun_out/r5_edges6_tests.log
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r5edges6_prof -o run -- python3 $ROOT/scripts/odd_sq.py 10 4096 x42,x83 > $ROOT/gpurun_out/r5edges6_prof.log 2>&1) || exit $?
