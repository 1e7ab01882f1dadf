#!/bin/bash
# GPU-box: stripe-plan / verify variants, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2 3; do
  for v in ${PLAN_VARIANTS:-base st8 st16 st32 vf8 vf16 vf32}; do
    HBEC_LIB=tune_build/plan_$v/libhbec.so TUNE_LABEL=$v timeout -k 10 120 python scripts/tune_plan.py || exit $?
  done
done
