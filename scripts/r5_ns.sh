#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bitplane.py tests/test_gpu_unaligned.py tests/test_gpu_random_plan.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_ns_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_ns_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1500 bash scripts/ab_odd.sh gpurun_out/r5_ab17.jsonl o53,o64,o102,o103,o122,o123,v53,v64,v102,v103,v122,v123,p102,p123,p64 tune_build/tune/libhbec.so:HBEC_ODD_BP=1 tune_build/tune/libhbec.so:HBEC_ODD_BP=0 || exit $?
