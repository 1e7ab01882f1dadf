#!/bin/bash
# Round-3 GPU batch 6: parity of gf_wide apply (k > 8 at any alignment) and
# plan U = 2, then gf_wide apply A/B against the round-2 kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py tests/test_gpu_parity.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b6_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b6_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd_env.sh $OUT/r3b6_tune_wide.jsonl "base:HBEC_WIDE_BPC=4" "base:HBEC_WIDE_BPC=8" "base:HBEC_WIDE_APPLY=0" || exit $?
echo done
