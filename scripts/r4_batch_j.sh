# round-4 batch J: LDS coefficient tables of the K >= 9 record kernels read by compiler-scheduled loads
bash scripts/ab_odd.sh gpurun_out/r4ab9.jsonl o104,o124,p104,p124,o83 hummingbird_amd/libhbec.so tune_build/odd_ldscc/libhbec.so
