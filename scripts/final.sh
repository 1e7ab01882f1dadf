#!/bin/bash
# A round's final measurements: whole GPU suite, smoke, PMC passes (the
# summary is written on the box and copied to profiles/ so the bench line
# below quotes it), bench line; `second`: a second bench line, rocprof stats
# of bench.py and SQ counters of the odd kernels.
# usage: scripts/final.sh [all|first|second]   (env TAG, default r06)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${TAG:-r06}
if [ "${1:-all}" = "second" ]; then
  timeout -k 10 500 python bench.py > $OUT/${T}_bench2.json 2> $OUT/${T}_bench2.err || exit 1
  tail -c 200 $OUT/${T}_bench2.json
  bash scripts/gpu_run.sh prof || exit 1
  bash scripts/sq_odd.sh ${T}final o42,o63,o83,o104,o124,v83,v104,v124,r83,r104,x83 > $OUT/${T}final_sq.log 2>&1 || exit 1
  echo second-done; exit 0
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${T}_tests.log 2>&1; rc=$?; tail -3 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || exit 1
tail -2 $OUT/${T}_smoke.log
bash scripts/gpu_run.sh pmcfetch pmcwrite || exit 1
python scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/${T}_pmc.json > /dev/null || exit 1
cp $OUT/${T}_pmc.json profiles/${T}_pmc.json
timeout -k 10 500 python bench.py > $OUT/${T}_bench.json 2> $OUT/${T}_bench.err || exit 1
tail -c 300 $OUT/${T}_bench.json
[ "${1:-all}" = "first" ] && { echo first-done; exit 0; }
bash scripts/gpu_run.sh prof || exit 1
bash scripts/sq_odd.sh ${T}final o42,o63,o83,o104,o124,v83,v104,v124,r83,r104,x83 > $OUT/${T}final_sq.log 2>&1 || exit 1
echo final-done
