#!/bin/bash
# GPU side of scripts/tune_unaligned.py: every variant, interleaved by process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base noclamp base noclamp; do
  HBEC_LIB=tune_build/unal_$v/libhbec.so timeout -k 10 120 python scripts/tune_unaligned.py run $v \
    >> gpurun_out/tune_unaligned.jsonl 2>> gpurun_out/tune_unaligned.err || exit $?
done
