#!/bin/bash
# round 5 A/B driver: scripts/r5_ab.sh OUT SHAPES LIB...  (each lib a path or path:VAR=VAL)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=$1; shift
timeout -k 10 1000 bash scripts/ab_odd.sh "gpurun_out/$out" "$@"
