#!/bin/bash
# Interleaved A/B of library builds on scripts/odd_sq.py shapes: one process
# per (round, library), libraries alternated, 3 rounds.
# usage: scripts/ab_odd.sh OUT.jsonl SHAPES LIB[:VAR=VAL[:VAR=VAL]] ...
set -u
out=$1; shapes=$2; shift 2
for r in 0 1 2; do
  for spec in "$@"; do
    IFS=: read -r lib envs <<< "$spec"
    envarr=()
    [ -n "${envs:-}" ] && IFS=: read -ra envarr <<< "$envs"
    env "${envarr[@]}" AB_ROUND=$r HBEC_LIB=$lib AB_LABEL="$spec" timeout -k 10 200 python scripts/odd_sq.py 15 ${AB_N:-2048} "$shapes" >> "$out" 2>> "${out%.jsonl}.err" || exit $?
  done
done
python - "$out" <<'PY'
import json, sys, statistics, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith("{"):
        r = json.loads(l); d[(r["shape"], r.get("label", r["lib"]))].append(r["frac"])
for (sh, lib), v in sorted(d.items()):
    print(f"{sh:6s} {lib:55s} median {statistics.median(v):.4f}  {v}")
PY
