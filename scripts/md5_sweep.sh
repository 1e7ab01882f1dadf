#!/bin/bash
# GPU-box: MD5 depth variants (tune_build/md5_d*/libhbec.so, built on the CPU
# side by `python scripts/md5_sweep_build.py`) and pipeline segment counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${MD5_VARIANTS:-}; do
  HBEC_LIB=tune_build/md5_$v/libhbec.so timeout -k 10 120 python scripts/bench_md5.py --no-cpu --label md5_$v || exit $?
done
for n in ${MD5_SEGMENTS:-}; do
  HBEC_MD5_SEGMENTS=$n timeout -k 10 120 python scripts/bench_md5.py --no-cpu --label seg$n || exit $?
done
