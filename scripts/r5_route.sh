#!/bin/bash
# The record-kernel route for 16-B-aligned views: GPU suite, then the product
# (route on) against the same library with HBEC_REC_ROUTE=0 (aligned kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_route_tests.log 2>&1 || { tail -30 gpurun_out/r5_route_tests.log; exit 1; }
tail -2 gpurun_out/r5_route_tests.log
SH=c:8:3:131088:enc,c:8:3:131120:enc,c:6:4:174768:enc,c:8:4:131088:enc,c:10:4:131072:enc,c:12:4:87424:enc,c:9:3:131072:enc,c:10:4:104864:rec,c:12:4:87424:rec,c:8:3:131088:rec,c:10:4:4096:enc,c:12:4:2048:enc,c:8:3:4112:enc,c:10:2:2064:enc,c:8:3:131072:enc,c:4:2:262160:enc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_route.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_REC_ROUTE=0 || exit $?
