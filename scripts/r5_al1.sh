#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
HBEC_LIB=$PWD/tune_build/aload/libhbec.so HBEC_ODD_BP=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_bitplane.py tests/test_gpu_unaligned.py tests/test_gpu_random_plan.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_al1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_al1_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab15.jsonl o83,o104,o124,o63,p83,o84 tune_build/aload/libhbec.so:HBEC_ODD_BP=2 tune_build/tune/libhbec.so:HBEC_ODD_BP=2 tune_build/tune/libhbec.so:HBEC_ODD_BP=0 || exit $?
