#!/bin/bash
# Round-3 GPU batch 5: gf_verify_wide parity + grid A/B, then the gf_odd variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unaligned.py -k verify -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b5_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b5_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 4 2 8; do
  HBEC_WIDE_BPC=$b timeout -k 10 200 python scripts/bench_verify_wide.py > $OUT/r3b5_verify_wide_bpc$b.jsonl 2>&1 || exit $?
done
bash scripts/r3_batch4.sh || exit $?
echo done
