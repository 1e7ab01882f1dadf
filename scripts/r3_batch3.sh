#!/bin/bash
# Round-3 GPU batch 3: parity of the new kernels (mirrored gf_odd plans,
# gf_verify_wide, accumulate prefetch), then wide Verify A/B and the pinned
# odd-size encode + ShardHash host bench.  Every step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b3_tests.log 2>&1
rc=$?; tail -5 $OUT/r3b3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/bench_verify_wide.py > $OUT/r3b3_verify_wide.jsonl 2>&1 || exit $?
HBEC_WIDE_VERIFY=0 timeout -k 10 200 python scripts/bench_verify_wide.py >> $OUT/r3b3_verify_wide.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_host_odd.py r3 4096 md5 > $OUT/r3b3_host_odd_md5.jsonl 2>&1 || exit $?
echo done
