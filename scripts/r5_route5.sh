#!/bin/bash
# Final record-kernel routing rule: GPU suite, then the rule against
# HBEC_REC_ROUTE=0 (every 16-B-aligned view on the aligned kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_route5_tests.log 2>&1 || { tail -40 gpurun_out/r5_route5_tests.log; exit 1; }
tail -2 gpurun_out/r5_route5_tests.log
SH=c:7:4:149888:enc,c:7:4:149904:enc,c:6:4:174848:enc,c:8:4:131072:plan,c:8:4:131072:dplan,c:6:4:174848:plan,c:6:6:174848:enc,c:8:3:131088:enc,c:10:4:131072:enc,c:12:4:87424:dplan,c:8:3:131072:enc,c:4:2:262144:enc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_route5.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_REC_ROUTE=0 || exit $?
