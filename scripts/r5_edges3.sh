#!/bin/bash
# Edge kernel before the main kernel (HBEC_EDGE_FIRST=1: its 73 MB of edge
# lines may still be in the Infinity Cache when the main kernel reads them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:8191:enc,c:4:2:4095:enc,c:8:3:16383:enc,c:8:3:8191:ver
AB_N=16384 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_edges3.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_EDGE_FIRST=1 || exit $?
SH=o83,o42,v83
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_edges3.jsonl $SH tune_build/va/libhbec.so tune_build/va/libhbec.so:HBEC_EDGE_FIRST=1 || exit $?
