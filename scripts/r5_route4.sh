#!/bin/bash
# 4 parity rows at 128-B pitches, 5 <= k <= 8: aligned / stripe kernels vs the
# record kernels (HBEC_REC_ROUTE=2), strided, stripe-plan and object-plan.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:6:4:174848:enc,c:8:4:131072:enc,c:5:4:209792:enc,c:7:4:149888:enc,c:6:4:174848:plan,c:8:4:131072:plan,c:8:4:131072:dplan,c:6:4:174848:dplan,c:8:5:131072:enc,c:6:6:174848:enc,c:8:3:131072:enc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_route4.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_REC_ROUTE=2 || exit $?
