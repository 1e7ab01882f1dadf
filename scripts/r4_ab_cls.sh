# round-4: plans of two odd size classes on per-class record launches vs gf_odd_plan (one class allowed)
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4q_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_odd.sh gpurun_out/r4ab12.jsonl c42,c83,c104,p124 hummingbird_amd/libhbec.so tune_build/odd_cls1/libhbec.so
bash scripts/ab_odd.sh gpurun_out/r4ab13.jsonl o63,o73,o62,o42 hummingbird_amd/libhbec.so tune_build/odd_rec18/libhbec.so
