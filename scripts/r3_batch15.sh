#!/bin/bash
# Round-3 GPU batch 15: PMC refresh + bench line on the current tree
# (scripts/r3_batch12.sh), then the cross-window carry parity and A/B
# (scripts/r3_batch14.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/r3_batch12.sh r3b15 || exit $?
bash scripts/r3_batch14.sh || exit $?
echo done
