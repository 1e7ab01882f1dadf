# round-4 batch F: GPU suite (many-tile odd shapes, near-uniform plans), odd-kernel A/B, MD5 pipeline variants
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4f_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_odd.sh gpurun_out/r4ab6.jsonl o42,r42,v42,o83,r83,v83,o104,r104,o124,p124 hummingbird_amd/libhbec.so tune_build/odd_r3/libhbec.so tune_build/odd_rec0/libhbec.so tune_build/odd_u0/libhbec.so tune_build/odd_l5/libhbec.so tune_build/odd_pf0/libhbec.so || exit 1
bash scripts/md5_pipe_sweep.sh gpurun_out/r4md5b.jsonl "HBEC_LIB=hummingbird_amd/libhbec.so" "HBEC_LIB=tune_build/odd_md5p/libhbec.so" "HBEC_LIB=tune_build/odd_md5d4/libhbec.so"
