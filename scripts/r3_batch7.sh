#!/bin/bash
# Round-3 GPU batch 7: parity after the odd.hip split (three translation
# units), then base vs K <= 12 gf_odd vs 16-B loads for K <= 4 vs wide ring depth 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py tests/test_gpu_parity.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b7_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b7_tests.log; [ $rc -eq 0 ] || exit $rc
HBEC_LIB=tune_build/odd_maxk12/libhbec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_unaligned.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b7_tests_maxk12.log 2>&1
rc=$?; tail -3 $OUT/r3b7_tests_maxk12.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd_env.sh $OUT/r3b7_tune.jsonl base maxk12 aload4 wd8 wu2 || exit $?
echo done
