#!/bin/bash
# Shard-length threshold of the record-kernel route for 16-B-aligned views.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:8208:enc,c:8:3:16400:enc,c:8:3:32784:enc,c:8:3:65552:enc,c:10:4:8192:enc,c:10:4:16384:enc,c:10:4:32768:enc,c:10:4:65536:enc,c:12:4:16384:enc,c:12:4:32768:enc,c:12:4:65536:enc,c:6:4:16400:enc,c:6:4:65552:enc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_route2.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_REC_ROUTE=0 || exit $?
