#!/bin/bash
# Routing policy for 16-B-aligned views: aligned kernels vs record kernels for
# 128-B-aligned pitches (k > 8 and k <= 8) and more non-128 pitches, encode and
# reconstruct.  HBEC_VEC_ALIGN=2^30 sends every view to the record kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:10:4:131072:enc,c:12:4:131072:enc,c:9:3:131072:enc,c:10:4:104960:enc,c:12:4:87424:enc,c:10:4:131072:rec,c:12:4:87424:rec,c:10:2:131072:enc,c:12:3:87424:enc
SH=$SH,c:8:3:131072:enc,c:6:3:174848:enc,c:4:2:262144:enc,c:8:3:131072:rec
SH=$SH,c:8:3:131104:enc,c:8:3:131120:enc,c:7:3:149808:enc,c:5:3:209728:enc,c:8:4:131088:enc,c:8:2:131088:enc,c:6:4:174768:enc,c:8:3:131088:rec,c:4:2:262160:rec
timeout -k 10 1100 bash scripts/ab_odd.sh gpurun_out/r5_va2.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_VEC_ALIGN=128 tune_build/va/libhbec.so:HBEC_VEC_ALIGN=1073741824 || exit $?
