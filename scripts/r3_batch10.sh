#!/bin/bash
# Round-3 GPU batch 10: windows per wave tile for 5 <= K <= 8 (gf_odd), A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/tune_odd_env.sh $OUT/r3b10_tune.jsonl base umid2 umid3 || exit $?
echo done
