#!/bin/bash
# GPU suite, then the Verify route (8+4 class) against HBEC_VERIFY_ROUTE=0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_vroute2_tests.log 2>&1 || { tail -40 gpurun_out/r5_vroute2_tests.log; exit 1; }
tail -2 gpurun_out/r5_vroute2_tests.log
SH=c:8:4:131072:ver,c:8:4:131088:ver,c:8:4:65536:ver,c:8:3:131072:ver,c:6:4:174848:ver,c:7:4:149888:ver
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_vroute2.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_VERIFY_ROUTE=0 || exit $?
