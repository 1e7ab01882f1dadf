#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1200 bash scripts/ab_odd.sh gpurun_out/r5_ab16.jsonl v83,v104,v124,v63,v84,v93,v73,v62,v82 tune_build/tune/libhbec.so:HBEC_ODD_BP=2 tune_build/vbar/libhbec.so:HBEC_ODD_BP=2 tune_build/tune/libhbec.so:HBEC_ODD_BP=1 || exit $?
HBEC_ODD_BP=2 bash scripts/r5_pmc_odd.sh r5pmcVB2 v83,v104,v124 tune_build/vbar/libhbec.so > /dev/null 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5pmcVB2_pmc.json"))["kernels"]
alg = {(8, 3): 2048*11*131071, (10, 4): 2048*14*104858, (12, 4): 2048*16*87389}
for k, v in d.items():
    if ", 2, " in k and "gf_odd_rec" in k:
        kk = tuple(int(x) for x in k.split("<")[1].split(",")[:2])
        print("vbar", k, v["hbm_read_bytes_per_launch"], round(v["hbm_read_bytes_per_launch"] / alg[kk], 4))
PY
