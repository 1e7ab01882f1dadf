#!/bin/bash
# Round-3 GPU batch 19: output columns pinned after the field multiply (K >= 5:
# 8+3 275 -> 201 VGPRs, 10+4 392 -> 267), alone and with 2 blocks per CU
# (launch bounds 2: 2 waves per SIMD).  Parity first with the 2-block library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
HBEC_LIB=tune_build/odd_pinlb2/libhbec.so HBEC_ODD_BPC=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py tests/test_gpu_parity.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b19_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b19_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd_env.sh $OUT/r3b19_tune.jsonl base pin pin:HBEC_ODD_BPC=2 pinlb2:HBEC_ODD_BPC=2 pinlb2 || exit $?
echo done
