#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_ab9.jsonl v83,v104,v42,v124 tune_build/tune/libhbec.so tune_build/vkeep/libhbec.so || exit $?
for L in tune vkeep; do
  bash scripts/r5_pmc_odd.sh r5pmcV$L v83,v104,v42 tune_build/$L/libhbec.so > /dev/null 2>&1 || exit $?
done
python - <<'PY'
import json
alg = {"gf_odd<8, 3, 2>": 2048*11*131071, "gf_odd_rec<10, 4, 2, -1>": 2048*14*104858, "gf_odd<4, 2, 2>": 2048*6*262143}
for t in ("tune", "vkeep"):
    d = json.load(open(f"gpurun_out/r5pmcV{t}_pmc.json"))["kernels"]
    for k, v in d.items():
        if k in alg:
            print(t, k, v["hbm_read_bytes_per_launch"], round(v["hbm_read_bytes_per_launch"] / alg[k], 4))
PY
