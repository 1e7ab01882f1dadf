#!/bin/bash
# round 5: first GPU run of the bit-plane record kernels: parity tests, then
# an interleaved A/B of the odd shapes against the round-4 library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bitplane.py tests/test_gpu_unaligned.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_bp1_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5_bp1_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 bash scripts/ab_odd.sh gpurun_out/r5_ab1.jsonl o83,o104,o124,o63,o73,o42,p83,p104 hummingbird_amd/libhbec.so tune_build/r4/libhbec.so
