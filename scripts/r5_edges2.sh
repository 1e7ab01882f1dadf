#!/bin/bash
# Edge kernel beside the main kernel (side stream): GPU suite, then the
# product against HBEC_EDGE_OVERLAP=0, short odd shards and 1-MiB-class ones.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_edges2_tests.log 2>&1 || { tail -40 gpurun_out/r5_edges2_tests.log; exit 1; }
tail -2 gpurun_out/r5_edges2_tests.log
SH=c:8:3:4095:enc,c:8:3:8191:enc,c:8:3:16383:enc,c:4:2:4095:enc,c:4:2:16383:enc,c:10:4:8191:enc,c:8:3:8191:ver,c:4:2:8191:rec
AB_N=16384 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_edges2.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_EDGE_OVERLAP=0 || exit $?
SH=o83,o42,o104,v83,v42,r83
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_edges2.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_EDGE_OVERLAP=0 || exit $?
