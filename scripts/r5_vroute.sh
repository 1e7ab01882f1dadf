#!/bin/bash
# Verify of 16-B-aligned views, 5 <= k <= 8: gf_verify_pipe vs the record
# kernels (HBEC_VERIFY_ROUTE 1: the apply rule, 2: every S >= 48 KiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:131072:ver,c:8:3:131088:ver,c:8:4:131072:ver,c:8:4:131088:ver,c:6:4:174848:ver,c:6:3:174768:ver,c:5:3:209728:ver,c:7:3:149808:ver,c:8:2:131088:ver,c:6:2:174768:ver
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_vroute.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_VERIFY_ROUTE=2 || exit $?
