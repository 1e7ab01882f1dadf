#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab8.jsonl o83,o104,o124,o63,p42b,p83 tune_build/tune/libhbec.so:HBEC_ODD_BP=2 tune_build/order0/libhbec.so:HBEC_ODD_BP=2 tune_build/tune/libhbec.so:HBEC_ODD_BP=0 tune_build/order0/libhbec.so:HBEC_ODD_BP=0 || exit $?
HBEC_ODD_BP=2 bash scripts/r5_pmc_odd.sh r5pmcB1 o83,o104 tune_build/tune/libhbec.so > /dev/null 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5pmcB1_pmc.json"))["kernels"]
for k, v in d.items():
    if "gf_odd_rec" in k:
        print("B1", k, v["hbm_read_bytes_per_launch"], v["hbm_write_bytes_per_launch"])
PY
