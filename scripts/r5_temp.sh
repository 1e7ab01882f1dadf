#!/bin/bash
# Temporal-hint input loads in the record kernels (HBEC_ODD_TEMP: 1 Verify,
# 3 Verify + apply) against the non-temporal tuning build: rate and reads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=v83,v104,v124,o83,o104,o124,p83,x83
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_temp.jsonl $SH tune_build/tune/libhbec.so tune_build/t1/libhbec.so tune_build/t3/libhbec.so || exit $?
for l in tune t3; do
  bash scripts/r5_pmc_odd.sh r5temp_$l v83,v104,o83,o104 tune_build/$l/libhbec.so > /dev/null 2>&1 || exit $?
done
python - <<'PY'
import json
alg = {(8, 3): 2048*11*131071, (10, 4): 2048*14*104858}
for l in ("tune", "t3"):
    d = json.load(open(f"gpurun_out/r5temp_{l}_pmc.json"))["kernels"]
    for k, v in d.items():
        if "gf_odd_rec" in k:
            kk = tuple(int(x) for x in k.split("<")[1].split(",")[:2])
            if kk in alg:
                print(l, k, v["hbm_read_bytes_per_launch"], round(v["hbm_read_bytes_per_launch"] / alg[kk], 4))
PY
