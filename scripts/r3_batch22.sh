#!/bin/bash
# Round-3 GPU batch 22: apply without the per-tile block barrier (Verify already
# runs without it) on top of the pinned-output default, all odd shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/tune_odd.sh $OUT/r3b22_tune.jsonl base nobar || exit $?
echo done
