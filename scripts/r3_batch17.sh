#!/bin/bash
# Round-3 GPU batch 17: 2 windows per tile (now with the carry) for 5 <= K <= 8,
# and a stripe plan of uniform odd stripes next to the mixed-size one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
HBEC_LIB=tune_build/odd_umid2/libhbec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_unaligned.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b17_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b17_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd_env.sh $OUT/r3b17_tune.jsonl base umid2 || exit $?
echo done
