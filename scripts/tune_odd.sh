#!/bin/bash
# Alternate the gf_odd variants' processes (scripts/tune_odd.py), 2 rounds.
# usage: scripts/tune_odd.sh OUT.jsonl variant...   (variant "base" = hummingbird_amd/libhbec.so)
set -u
out=$1; shift
for r in 0 1; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=hummingbird_amd/libhbec.so; else lib=tune_build/odd_$v/libhbec.so; fi
    HBEC_ODD=1 HBEC_LIB=$lib timeout -k 10 240 python scripts/tune_odd.py run "$v" "$r" >> "$out" 2>&1 || exit $?
  done
done
