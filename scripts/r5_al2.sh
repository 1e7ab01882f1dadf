#!/bin/bash
# 16-B-aligned shard pitches that are not multiples of the 128-B line: rate and
# reads of the aligned kernels (8+3, 4+2, 10+4 databuf encode).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:131072:enc,c:8:3:131088:enc,c:8:3:131136:enc,c:8:3:131200:enc,c:4:2:262144:enc,c:4:2:262160:enc,c:4:2:262208:enc,c:10:4:104960:enc,c:10:4:104864:enc
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_al2.jsonl $SH hummingbird_amd/libhbec.so || exit $?
bash scripts/r5_pmc_odd.sh r5al2 $SH hummingbird_amd/libhbec.so > /dev/null 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5al2_pmc.json"))
print(json.dumps(d, indent=0)[:6000])
PY
