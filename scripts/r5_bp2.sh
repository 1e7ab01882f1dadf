#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bitplane.py tests/test_gpu_unaligned.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_bp2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_bp2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab7.jsonl o82,o84,o93,o62,p63,p73,p42b,o124,o104 hummingbird_amd/libhbec.so tune_build/tune/libhbec.so:HBEC_ODD_BP=2 tune_build/tune/libhbec.so:HBEC_ODD_BP=0 || exit $?
bash scripts/r5_pmc_odd.sh r5pmcT o83 tune_build/tune/libhbec.so > /dev/null 2>&1 || exit $?
HBEC_ODD_BP=2 bash scripts/r5_pmc_odd.sh r5pmcB o83 tune_build/tune/libhbec.so > /dev/null 2>&1 || exit $?
python - <<'PY'
import json
for t in ("T", "B"):
    d = json.load(open(f"gpurun_out/r5pmc{t}_pmc.json"))["kernels"]
    for k, v in d.items():
        if "gf_odd_rec" in k:
            print(t, k, v["hbm_read_bytes_per_launch"], v["hbm_write_bytes_per_launch"])
PY
