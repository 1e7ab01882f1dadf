#!/bin/bash
# Round-3 GPU batch 11: the whole -m gpu suite (no -x), then the U-mid A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 780 python -u -m pytest tests -m gpu -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests_all.log 2>&1
rc=$?; tail -12 $OUT/tests_all.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r3_batch10.sh || exit $?
echo done
