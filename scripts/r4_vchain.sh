# round-4: odd Verify windows (K <= 4): chained 64 U - 1 columns per tile vs 63 per window; speed A/B, then FETCH_SIZE per library
set -u
ROOT=$(cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && pwd)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$ROOT/gpurun_out; export TMPDIR=/tmp
HBEC_LIB=tune_build/odd_vc4/libhbec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_unaligned.py -q -k "verify" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r4v_tests.log 2>&1; rc=$?; tail -2 $OUT/r4v_tests.log; [ $rc -eq 0 ] || exit 1
HBEC_LIB=tune_build/odd_vc2/libhbec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_unaligned.py -q -k "verify" --timeout 120 --timeout-method thread -p no:cacheprovider >> $OUT/r4v_tests.log 2>&1; rc=$?; tail -2 $OUT/r4v_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_odd.sh $OUT/r4ab16.jsonl v42,v32 hummingbird_amd/libhbec.so tune_build/odd_vc2/libhbec.so tune_build/odd_vc4/libhbec.so tune_build/odd_vu4/libhbec.so || exit 1
for lib in hummingbird_amd tune_build/odd_vc2 tune_build/odd_vc4 tune_build/odd_vu4; do
  tag=$(echo $lib | tr '/' '_')
  mkdir -p $OUT/vpmc_$tag
  (cd /tmp && HBEC_LIB=$ROOT/$lib/libhbec.so timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/vpmc_$tag -o run -- python3 $ROOT/scripts/odd_sq.py 3 2048 v42 > $OUT/vpmc_$tag.log 2>&1) || exit 1
done
echo done
