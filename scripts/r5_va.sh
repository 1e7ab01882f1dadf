#!/bin/bash
# 16-B-aligned views that are not 128-B aligned: aligned kernels (default) vs
# the record kernels (tuning knob HBEC_VEC_ALIGN=128 routes them to gf_odd).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:131088:enc,c:8:3:131136:enc,c:8:3:131152:enc,c:8:3:131200:enc,w:8:3:131072:16:0,w:8:3:131072:0:16,w:8:3:131072:16:16,c:4:2:262160:enc,c:4:2:262208:enc,c:6:3:174768:enc,c:10:4:104864:enc,c:12:4:87392:enc,c:8:3:131088:ver,c:4:2:262160:ver
timeout -k 10 1000 bash scripts/ab_odd.sh gpurun_out/r5_va.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_VEC_ALIGN=128 || exit $?
