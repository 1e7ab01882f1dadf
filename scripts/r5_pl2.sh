#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bitplane.py tests/test_gpu_unaligned.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_pl2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_pl2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab12.jsonl p83,p104,p42b,c83,c104,c42,o104,o83 hummingbird_amd/libhbec.so tune_build/tune/libhbec.so || exit $?
AB_N=4096 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab13.jsonl x42,x83,x104 hummingbird_amd/libhbec.so tune_build/tune/libhbec.so || exit $?
