#!/bin/bash
# Headline grid re-check with the tuning build's runtime knobs: blocks per CU
# (1 shipped, 2) and tiles per launch (1 Mi shipped, 256 Ki, 4 Mi).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
L=tune_build/tune/libhbec.so
AB_N=4096 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_grid.jsonl a42,c:4:2:262144:rec $L $L:HBEC_BLOCKS_PER_CU=2 $L:HBEC_CHUNK_TILES=262144 $L:HBEC_CHUNK_TILES=4194304 || exit $?
