#!/bin/bash
# Round-3 GPU batch 16: the carry as default (strided + plans with K <= 4):
# parity of every unaligned path, one tune_odd round, then the PMC refresh and
# bench line (scripts/r3_batch12.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py tests/test_gpu_databuf.py tests/test_gpu_ecstream.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_large.py tests/test_gpu_rings.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b16_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b16_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python scripts/tune_odd.py run base 0 > $OUT/r3b16_tune.jsonl 2>&1 || exit $?
bash scripts/r3_batch12.sh r3b16 || exit $?
echo done
