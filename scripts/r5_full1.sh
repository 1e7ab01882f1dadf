#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -x > gpurun_out/r5_full1_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5_full1_tests.log; exit $rc
