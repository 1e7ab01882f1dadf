#!/bin/bash
# Edge kernel with 64 + 64 slots for long shards: GPU suite, traces of 16384
# short objects (8+3, 4+2) and of one-object calls, and the odd legs' rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_edges5_tests.log 2>&1 || { tail -40 gpurun_out/r5_edges5_tests.log; exit 1; }
tail -2 gpurun_out/r5_edges5_tests.log
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r5edges5_prof -o run -- python3 $ROOT/scripts/odd_sq.py 10 16384 c:8:3:8191:enc,c:4:2:4095:enc,c:8:3:8191:ver > $ROOT/gpurun_out/r5edges5_prof.log 2>&1) || exit $?
SH=c:8:3:8191:enc,c:4:2:4095:enc,c:8:3:16383:enc,c:8:3:8191:ver
AB_N=16384 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_edges5.jsonl $SH hummingbird_amd/libhbec.so || exit $?
