#!/bin/bash
# round-5 final measurements: whole GPU suite, smoke, PMC passes (summary
# written on the box so the bench line below quotes it), bench line, rocprof
# stats, SQ counters of the odd kernels (this library and the round-4 one)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${1:-all}" = "second" ]; then
  timeout -k 10 500 python bench.py > $OUT/r5l_bench2.json 2> $OUT/r5l_bench2.err || exit 1
  tail -c 200 $OUT/r5l_bench2.json
  bash scripts/gpu_run.sh prof || exit 1
  bash scripts/r5_sq.sh r5final o42,o63,o83,o104,o124,v83,v104,v124,r83,x83 > $OUT/r5final_sq.log 2>&1 || exit 1
  bash scripts/r5_sq.sh r5r4lib o63,o104,o124,v83,v104,v124 tune_build/r4/libhbec.so > $OUT/r5r4lib_sq.log 2>&1 || exit 1
  echo second-done; exit 0
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r5l_tests.log 2>&1; rc=$?; tail -3 $OUT/r5l_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r5l_smoke.log 2>&1 || exit 1
tail -2 $OUT/r5l_smoke.log
bash scripts/gpu_run.sh pmcfetch pmcwrite || exit 1
python scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/r05_pmc.json > /dev/null || exit 1
cp $OUT/r05_pmc.json profiles/r05_pmc.json
timeout -k 10 500 python bench.py > $OUT/r5l_bench.json 2> $OUT/r5l_bench.err || exit 1
tail -c 300 $OUT/r5l_bench.json
[ "${1:-all}" = "first" ] && { echo first-done; exit 0; }
bash scripts/gpu_run.sh prof || exit 1
bash scripts/r5_sq.sh r5final o42,o63,o83,o104,o124,v83,v104,v124,r83,x83 > $OUT/r5final_sq.log 2>&1 || exit 1
bash scripts/r5_sq.sh r5r4lib o63,o104,o124,v83,v104,v124 tune_build/r4/libhbec.so > $OUT/r5r4lib_sq.log 2>&1 || exit 1
echo final-done
