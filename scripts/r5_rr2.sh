#!/bin/bash
# 9 <= k <= 12 with 2 outputs (reconstruct of two shards, 10+2 / 12+2 tails):
# gf_odd (register tables) vs the record kernel (LDS tables), HBEC_ODD_REC_BIGK_MINR=2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=r104,c:12:4:87389:rec,c:9:3:116509:rec,c:10:2:104858:rec,c:11:3:95326:rec,o104
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_rr2.jsonl $SH tune_build/tune/libhbec.so tune_build/rr2/libhbec.so || exit $?
