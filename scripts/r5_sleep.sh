#!/bin/bash
# Headline kernel pacing re-check: gf_apply_vec_pipe2 s_sleep 4 / 6 / 8 (shipped) / 10
# after each tile's loads, 4096 x 1 MiB 4+2 encode and reconstruct {0,1}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
AB_N=4096 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_sleep.jsonl a42,c:4:2:262144:rec tune_build/s8/libhbec.so tune_build/s4/libhbec.so tune_build/s6/libhbec.so tune_build/s10/libhbec.so || exit $?
