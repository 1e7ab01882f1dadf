#!/bin/bash
# Round-3 GPU batch 4: gf_odd variant A/B (scripts/tune_odd.py, processes
# alternated, 2 rounds), each run under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
[ $# -gt 0 ] || set -- base aload edge ntst0 planu2 maxk12
bash scripts/tune_odd_env.sh $OUT/r3b4_tune_odd.jsonl "$@" || exit $?
echo done
