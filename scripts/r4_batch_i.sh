# round-4 batch I: odd 5 <= K <= 8 tiles (windows per wave tile, 2 waves per SIMD, LDS tables with 2 windows)
bash scripts/ab_odd.sh gpurun_out/r4ab8.jsonl o83,r83,v83,p83,o42,o104 hummingbird_amd/libhbec.so tune_build/odd_lb2/libhbec.so tune_build/odd_umid2/libhbec.so tune_build/odd_umid3/libhbec.so tune_build/odd_l5u2/libhbec.so
