#!/bin/bash
# Round-3 GPU batch 24: 2-block pinned apply extended to 8 <= K <= 10 with
# K * R >= 24 (8+3 encode / plans): the whole -m gpu suite, then the odd shapes
# against the previous default (tune_build/odd_prev).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b24_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b24_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd.sh $OUT/r3b24_tune.jsonl base prev || exit $?
echo done
