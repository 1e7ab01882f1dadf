#!/bin/bash
# Round-3 GPU batch 13: gf_odd Verify with 63-column windows (parity + A/B via
# tune_odd base runs), and gf_verify_wide ring depth / windows for 32+8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_pinning.py tests/test_gpu_packed.py -x -q --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3b13_tests.log 2>&1
rc=$?; tail -3 $OUT/r3b13_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 0 1; do
  timeout -k 10 240 python scripts/tune_odd.py run base $r >> $OUT/r3b13_tune.jsonl 2>&1 || exit $?
  for v in base wu1d8 wd8u2; do
    if [ $v = base ]; then lib=hummingbird_amd/libhbec.so; else lib=tune_build/odd_$v/libhbec.so; fi
    HBEC_LIB=$lib timeout -k 10 200 python scripts/bench_verify_wide.py > $OUT/r3b13_vw_${v}_$r.jsonl 2>&1 || exit $?
  done
done
echo done
