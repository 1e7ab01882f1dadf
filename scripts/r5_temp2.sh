#!/bin/bash
# Temporal-hint apply loads for the window-major (3-wave, 12+4) bit-plane kernels only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_temp2.jsonl o124,p124,x124,o104,o83 tune_build/tune/libhbec.so tune_build/t4/libhbec.so || exit $?
for l in tune t4; do
  bash scripts/r5_pmc_odd.sh r5temp2_$l o124,p124 tune_build/$l/libhbec.so > /dev/null 2>&1 || exit $?
done
python - <<'PY'
import json
for l in ("tune", "t4"):
    d = json.load(open(f"gpurun_out/r5temp2_{l}_pmc.json"))["kernels"]
    for k, v in d.items():
        if "gf_odd_rec" in k:
            print(l, k, v["hbm_read_bytes_per_launch"], v.get("hbm_write_bytes_per_launch"), 2048*12*87389, 2048*12*87392)
PY
