# round-4 batch E: GPU suite, odd-kernel A/B (records: unrolled / not, LDS tables from K = 5), MD5 pipeline variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_odd.sh gpurun_out/r4ab5.jsonl o42,r42,v42,o83,r83,v83,o104,r104,o124,p124 tune_build/odd_r3/libhbec.so hummingbird_amd/libhbec.so tune_build/odd_u0/libhbec.so tune_build/odd_l5/libhbec.so tune_build/odd_l5u0/libhbec.so || exit 1
bash scripts/md5_pipe_sweep.sh gpurun_out/r4md5b.jsonl "HBEC_LIB=hummingbird_amd/libhbec.so" "HBEC_LIB=tune_build/odd_md5p/libhbec.so" "HBEC_LIB=tune_build/odd_md5d4/libhbec.so"
