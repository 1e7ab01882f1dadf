# round-4: LDS coefficient tables (compiler-scheduled reads) from K = 5 vs register tables for 5 <= K <= 8
bash scripts/ab_odd.sh gpurun_out/r4ab11.jsonl o83,p83,v83,o42 hummingbird_amd/libhbec.so tune_build/odd_l5/libhbec.so
