#!/bin/bash
# Aligned kernels at 16-B-aligned shard pitches that are not multiples of the
# 128-B line: product vs pipe2 (block barrier) for K <= 8, temporal-hint loads,
# input-major loads; reads from FETCH_SIZE for the product and the temporal build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:131072:enc,c:8:3:131088:enc,c:8:3:131136:enc,c:8:3:131200:enc,c:6:3:174768:enc,c:4:2:262144:enc,c:4:2:262160:enc,c:10:4:104864:enc
timeout -k 10 1000 bash scripts/ab_odd.sh gpurun_out/r5_al3.jsonl $SH hummingbird_amd/libhbec.so tune_build/pv2/libhbec.so tune_build/pt/libhbec.so tune_build/pi/libhbec.so tune_build/pv2i/libhbec.so || exit $?
for l in pt; do
  bash scripts/r5_pmc_odd.sh r5al3_$l $SH tune_build/$l/libhbec.so > /dev/null 2>&1 || exit $?
done
bash scripts/r5_pmc_odd.sh r5al3_prod $SH hummingbird_amd/libhbec.so > /dev/null 2>&1 || exit $?
