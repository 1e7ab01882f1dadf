# round-4 batch G: GPU suite, per-shape odd kernel policy + plan-record A/B, bench line
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4g_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_odd.sh gpurun_out/r4ab7.jsonl o42,r42,v42,o83,r83,v83,o104,r104,o124,p42,p83,p104,p124 hummingbird_amd/libhbec.so tune_build/odd_r3/libhbec.so tune_build/odd_pr24/libhbec.so tune_build/odd_pr99/libhbec.so || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err; tail -c 600 gpurun_out/r4g_bench.json
