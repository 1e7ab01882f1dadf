#!/bin/bash
# Bit-plane Verify of 10+4 / 12+4 at 2-3 blocks per CU (HBEC_ODD_BPC; the
# kernel holds 156 / 180 VGPRs): rate, and FETCH_SIZE per library setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_vbpc.jsonl v104,v124,v83 tune_build/tune/libhbec.so tune_build/tune/libhbec.so:HBEC_ODD_BPC=2 tune_build/tune/libhbec.so:HBEC_ODD_BPC=3 || exit $?
for b in 1 2 3; do
  HBEC_ODD_BPC=$b bash scripts/r5_pmc_odd.sh r5vbpc$b v104,v124 tune_build/tune/libhbec.so > /dev/null 2>&1 || exit $?
done
python - <<'PY'
import json
alg = {(10, 4): 2048*14*104858, (12, 4): 2048*16*87389}
for b in (1, 2, 3):
    d = json.load(open(f"gpurun_out/r5vbpc{b}_pmc.json"))["kernels"]
    for k, v in d.items():
        if "gf_odd_rec" in k and ", 2, " in k:
            kk = tuple(int(x) for x in k.split("<")[1].split(",")[:2])
            if kk in alg: print(b, k, round(v["hbm_read_bytes_per_launch"] / alg[kk], 4))
PY
