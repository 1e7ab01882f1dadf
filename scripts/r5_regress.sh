#!/bin/bash
# The current library against the one before this session's edge-kernel and
# 12 x 2 record changes (5fd2ec3), interleaved on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=v124,v104,v83,v42,o124,o104,o83,o42,r104,c:12:4:87389:rec,x83,x42
timeout -k 10 1000 bash scripts/ab_odd.sh gpurun_out/r5_regress.jsonl $SH hummingbird_amd/libhbec.so tune_build/pre_edges/libhbec.so || exit $?
