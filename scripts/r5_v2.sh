#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
HBEC_LIB=$PWD/tune_build/tune/libhbec.so HBEC_ODD_BP=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_unaligned.py -m gpu -x -q -k verify --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_v2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_v2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab14.jsonl v83,v104,v124,v63,v42 tune_build/tune/libhbec.so:HBEC_ODD_BP=2 tune_build/tune/libhbec.so:HBEC_ODD_BP=1 || exit $?
HBEC_ODD_BP=2 bash scripts/r5_pmc_odd.sh r5pmcVB v83,v104,v124,v63,v42 tune_build/tune/libhbec.so > /dev/null 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5pmcVB_pmc.json"))["kernels"]
alg = {(8, 3): 2048*11*131071, (10, 4): 2048*14*104858, (12, 4): 2048*16*87389, (6, 3): 2048*9*174763, (4, 2): 2048*6*262143}
for k, v in d.items():
    if ", 2, " in k and "gf_odd_rec" in k:
        kk = tuple(int(x) for x in k.split("<")[1].split(",")[:2])
        print(k, v["hbm_read_bytes_per_launch"], round(v["hbm_read_bytes_per_launch"] / alg[kk], 4))
PY
