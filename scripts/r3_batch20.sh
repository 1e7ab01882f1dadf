#!/bin/bash
# Round-3 GPU batch 20: the pinned-output policy as the default (Verify
# 5 <= K <= 8; 10+4-class apply with 2 blocks per CU): the whole -m gpu suite,
# then the odd tuning shapes (2 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b20_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b20_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd.sh $OUT/r3b20_tune.jsonl base || exit $?
echo done
