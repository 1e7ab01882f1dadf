#!/bin/bash
# Short odd shards (S = 4-16 KiB, 16384 objects) against their aligned
# neighbours: record / strided odd kernels vs the aligned ones; plus a
# rocprof kernel trace of the odd 8+3 S = 8191 encode (main vs edge kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
SH=c:8:3:4095:enc,c:8:3:4096:enc,c:8:3:8191:enc,c:8:3:8192:enc,c:8:3:16383:enc,c:8:3:16384:enc,c:4:2:4095:enc,c:4:2:4096:enc,c:4:2:16383:enc,c:4:2:16384:enc,c:10:4:8191:enc,c:10:4:8192:enc,c:8:3:8191:ver,c:8:3:8192:ver
AB_N=16384 timeout -k 10 900 bash scripts/ab_odd.sh gpurun_out/r5_small.jsonl $SH hummingbird_amd/libhbec.so || exit $?
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r5small_prof -o run -- python3 $ROOT/scripts/odd_sq.py 10 16384 c:8:3:8191:enc,c:4:2:4095:enc > $ROOT/gpurun_out/r5small_prof.log 2>&1) || exit $?
