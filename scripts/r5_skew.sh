#!/bin/bash
# Which side sets the aligned kernel's pitch sensitivity: inputs at i (S + DI),
# parity in its own array at r (S + DO), 8+3, S = 2^17 (w:K:M:S:DI:DO shapes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
SH=w:8:3:131072:0:0,w:8:3:131072:16:0,w:8:3:131072:0:16,w:8:3:131072:16:16,w:8:3:131072:64:0,w:8:3:131072:0:64,w:8:3:131072:128:0,w:8:3:131072:0:128,w:8:3:131072:16:128,w:8:3:131072:128:16,w:4:2:262144:0:16,w:4:2:262144:16:0
timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_skew.jsonl $SH hummingbird_amd/libhbec.so || exit $?
