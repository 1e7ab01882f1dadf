#!/bin/bash
# Round-3 GPU batch 8: parity with K <= 12 gf_odd, per-K plan tiles, wide U = 2
# and the new routing; then the odd-shape A/B, wide Verify / apply and k > 8 object plans.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py tests/test_gpu_parity.py tests/test_gpu_ecstream.py tests/test_gpu_databuf.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b8_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python scripts/tune_odd.py run base 0 > $OUT/r3b8_tune.jsonl 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_verify_wide.py > $OUT/r3b8_verify_wide.jsonl 2>&1 || exit $?
HBEC_WIDE_APPLY=0 timeout -k 10 200 python scripts/bench_verify_wide.py >> $OUT/r3b8_verify_wide.jsonl 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_objplan_wide.py > $OUT/r3b8_objplan_wide.jsonl 2>&1 || exit $?
timeout -k 10 240 python scripts/tune_odd.py run base 1 >> $OUT/r3b8_tune.jsonl 2>&1 || exit $?
echo done
