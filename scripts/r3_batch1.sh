#!/bin/bash
# Round-3 GPU batch: buffer OOB probe, gf_odd parity tests, gf_odd A/B, soak-stall reproduction.
set -u
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/oob_probe.bin > gpurun_out/r3_oob_probe.json 2>&1 || exit $?
HBEC_ODD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_ecstream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_odd_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_odd_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tune_odd_env.sh gpurun_out/r3_tune_odd3.jsonl "base:HBEC_ODD_BPC=1" "base:HBEC_ODD_BPC=2" "base:HBEC_ODD_BPC=4" \
  "u2:HBEC_ODD_BPC=1" "uv4:HBEC_ODD_BPC=1" "nobar:HBEC_ODD_BPC=1" "sleep:HBEC_ODD_BPC=1" "base:HBEC_ODD=0" || exit $?
timeout -k 10 150 ./scripts/soak_prefix.bin 64 100 > gpurun_out/r3_soak_prefix.jsonl 2> gpurun_out/r3_soak_prefix.err
echo "prefix rc=$?" >> gpurun_out/r3_soak_prefix.err
timeout -k 10 120 ./scripts/soak_cur.bin 64 60 > gpurun_out/r3_soak_cur.jsonl 2> gpurun_out/r3_soak_cur.err
echo "cur rc=$?" >> gpurun_out/r3_soak_cur.err
