#!/bin/bash
# Round-3 GPU batch 18: plan ids as scalars (no LDS-promoted record copies in
# gf_odd_plan): parity of every plan / zero-copy test, then the odd tuning
# shapes against the previous tree's library (tune_build/odd_oldplan).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_md5.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_packed.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b18_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b18_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd.sh $OUT/r3b18_tune.jsonl base oldplan || exit $?
echo done
