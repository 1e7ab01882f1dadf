# round-4 final measurements: whole GPU suite, smoke, PMC passes (summary written
# on the box so the bench line below quotes it), bench line, rocprof stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r4l_tests.log 2>&1; rc=$?; tail -3 $OUT/r4l_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r4l_smoke.log 2>&1 || exit 1
tail -2 $OUT/r4l_smoke.log
bash scripts/gpu_run.sh pmcfetch pmcwrite || exit 1
python scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/r04_pmc.json > /dev/null || exit 1
cp $OUT/r04_pmc.json profiles/r04_pmc.json
timeout -k 10 500 python bench.py > $OUT/r4l_bench.json 2> $OUT/r4l_bench.err || exit 1
tail -c 400 $OUT/r4l_bench.json
bash scripts/gpu_run.sh prof || exit 1
bash scripts/r4_sq.sh r4final o42,v42,o63,o83,v83,r83,o104,v104,o124,p42,p124 > gpurun_out/r4final_sq.log 2>&1 || exit 1
