#!/bin/bash
# Alternate (variant, env) runs of scripts/tune_odd.py, 2 rounds.
# usage: scripts/tune_odd_env.sh OUT.jsonl "variant:VAR=val" ...   (variant base = the in-tree library)
set -u
out=$1; shift
for r in 0 1; do
  for spec in "$@"; do
    v=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
    if [ "$v" = base ]; then lib=hummingbird_amd/libhbec.so; else lib=tune_build/odd_$v/libhbec.so; fi
    env HBEC_ODD=1 HBEC_LIB=$lib $envs timeout -k 10 240 python scripts/tune_odd.py run "$spec" "$r" >> "$out" 2>&1 || exit $?
  done
done
