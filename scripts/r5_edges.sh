#!/bin/bash
# Edge kernel, one thread per (object, slot) for all outputs: GPU suite, then
# short odd shards (16384 objects) and a kernel trace of 8+3 S = 8191.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_edges_tests.log 2>&1 || { tail -40 gpurun_out/r5_edges_tests.log; exit 1; }
tail -2 gpurun_out/r5_edges_tests.log
SH=c:8:3:4095:enc,c:8:3:8191:enc,c:8:3:16383:enc,c:4:2:4095:enc,c:4:2:16383:enc,c:10:4:8191:enc,c:8:3:8191:ver,c:8:3:131071:enc
AB_N=16384 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_edges.jsonl $SH hummingbird_amd/libhbec.so || exit $?
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r5edges_prof -o run -- python3 $ROOT/scripts/odd_sq.py 10 16384 c:8:3:8191:enc,c:4:2:4095:enc > $ROOT/gpurun_out/r5edges_prof.log 2>&1) || exit $?
