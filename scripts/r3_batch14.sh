#!/bin/bash
# Round-3 GPU batch 14: gf_odd cross-window carry (HBEC_ODD_CARRY=1 build):
# parity through the carry library, then the A/B against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
HBEC_LIB=tune_build/odd_carry/libhbec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_ecstream.py tests/test_gpu_databuf.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b14_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b14_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd_env.sh $OUT/r3b14_tune.jsonl base carry || exit $?
bash scripts/tune_odd_env.sh $OUT/r3b14_tune.jsonl base carry || exit $?
echo done
