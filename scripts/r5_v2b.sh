#!/bin/bash
# Bit-plane Verify at 2 blocks per CU with the per-tile block barrier for
# K R <= 40 (10+4) / 48 (12+4) instead of <= 27: rate and FETCH_SIZE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_v2b.jsonl v104,v124,v83 tune_build/tune/libhbec.so tune_build/v40/libhbec.so tune_build/v48/libhbec.so || exit $?
for l in tune v40 v48; do
  bash scripts/r5_pmc_odd.sh r5v2b_$l v104,v124 tune_build/$l/libhbec.so > /dev/null 2>&1 || exit $?
done
python - <<'PY'
import json
alg = {(10, 4): 2048*14*104858, (12, 4): 2048*16*87389}
for l in ("tune", "v40", "v48"):
    d = json.load(open(f"gpurun_out/r5v2b_{l}_pmc.json"))["kernels"]
    for k, v in d.items():
        if "gf_odd_rec" in k and ", 2, " in k:
            kk = tuple(int(x) for x in k.split("<")[1].split(",")[:2])
            if kk in alg: print(l, k, round(v["hbm_read_bytes_per_launch"] / alg[kk], 4))
PY
