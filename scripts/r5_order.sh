#!/bin/bash
# Does the order objects are coded in matter?  Databuf objects through an
# object plan in address order vs interleaved halves (0, n/2, 1, n/2+1, ...).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:131071:dplan,c:8:3:131071:dplanp,c:4:2:262143:dplan,c:4:2:262143:dplanp,c:10:4:104858:dplan,c:10:4:104858:dplanp,c:8:3:131072:dplan,c:8:3:131072:dplanp
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_order.jsonl $SH hummingbird_amd/libhbec.so || exit $?
