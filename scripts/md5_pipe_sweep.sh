#!/bin/bash
# Encode + ShardHash pipeline knobs (HBEC_MD5_*), one process per setting,
# settings alternated over 2 rounds.  usage: scripts/md5_pipe_sweep.sh OUT.jsonl "ENVS" ...
set -u
out=$1; shift
for r in 0 1; do
  for spec in "$@"; do
    env $spec AB_ROUND=$r timeout -k 10 120 python scripts/md5_pipe.py >> "$out" 2>> "${out%.jsonl}.err" || exit $?
  done
done
