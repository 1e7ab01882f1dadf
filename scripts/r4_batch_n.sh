# round-4 batch N: Verify of 9 <= k <= 12 through the record kernel (LDS tables) vs gf_verify_wide
HBEC_LIB=tune_build/odd_vk12/libhbec.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "verify or Verify" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4n_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4n_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_odd.sh gpurun_out/r4ab10.jsonl v104,v124,v83 hummingbird_amd/libhbec.so tune_build/odd_vk12/libhbec.so
