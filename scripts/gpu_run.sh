#!/bin/bash
# GPU-box runner: each step under its own time limit; stop at the first step
# that ends in anything but success / ordinary test failure (rc 0 or 1).
# usage: scripts/gpu_run.sh STEP [STEP ...]   (steps: tests smoke bench prof pmcfetch pmcwrite cfgprof cfgpmcfetch cfgpmcwrite ...)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a "$OUT/status.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/status.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a "$OUT/status.log"
    exit $rc
  fi
}
for s in "$@"; do
  case $s in
    build) step build 600 python -c "import __graft_entry__ as g; g.build()" ;;
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    testsall) step testsall 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 50 --warmup 10 ;;
    prof)
      mkdir -p "$OUT/prof"
      (cd /tmp && step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 10 --no-cpu-baseline --no-host-path --config5-objects 0) || exit $?
      ;;
    pmcfetch)
      mkdir -p "$OUT/pmc_fetch"
      (cd /tmp && step pmcfetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --config5-objects 0) || exit $?
      ;;
    pmcwrite)
      mkdir -p "$OUT/pmc_write"
      (cd /tmp && step pmcwrite 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --config5-objects 0) || exit $?
      ;;
    cfgprof)
      mkdir -p "$OUT/cfgprof"
      (cd /tmp && step cfgprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/cfgprof" -o run -- python3 "$ROOT/scripts/bench_configs.py") || exit $?
      ;;
    cfgpmcfetch)
      mkdir -p "$OUT/cfg_pmc_fetch"
      (cd /tmp && step cfgpmcfetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/cfg_pmc_fetch" -o run -- python3 "$ROOT/scripts/bench_configs.py") || exit $?
      ;;
    cfgpmcwrite)
      mkdir -p "$OUT/cfg_pmc_write"
      (cd /tmp && step cfgpmcwrite 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/cfg_pmc_write" -o run -- python3 "$ROOT/scripts/bench_configs.py") || exit $?
      ;;
    smallprof)
      mkdir -p "$OUT/smallprof"
      (cd /tmp && step smallprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/smallprof" -o run -- python3 "$ROOT/scripts/bench_small.py") || exit $?
      ;;
    smallpmcfetch)
      mkdir -p "$OUT/small_pmc_fetch"
      (cd /tmp && step smallpmcfetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/small_pmc_fetch" -o run -- python3 "$ROOT/scripts/bench_small.py") || exit $?
      ;;
    smallpmcwrite)
      mkdir -p "$OUT/small_pmc_write"
      (cd /tmp && step smallpmcwrite 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/small_pmc_write" -o run -- python3 "$ROOT/scripts/bench_small.py") || exit $?
      ;;
    small) step small 300 python scripts/bench_small.py ;;
    dist2) step dist2 600 env HBEC_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --objects 2048 ;;
    configs) step configs 600 python scripts/bench_configs.py ;;
    host) step host 600 python scripts/bench_host.py ;;
    ecloops)
      gcc -O2 -std=c11 -Iinclude scripts/bench_ecutils.c -Lhummingbird_amd -lhbec -Wl,-rpath,$ROOT/hummingbird_amd -o $OUT/bench_ecutils && step ecloops 300 sh -c "$OUT/bench_ecutils 4 2 256 && $OUT/bench_ecutils 8 3 256" ;;
    batcher)
      gcc -O2 -std=c11 -pthread -Iinclude scripts/bench_batcher.c -Lhummingbird_amd -lhbec -Wl,-rpath,$ROOT/hummingbird_amd -o $OUT/bench_batcher && step batcher 300 sh -c "for w in 1 2 3; do HBEC_BATCHER_WORKERS=\$w $OUT/bench_batcher 64 32 1 96 300 && HBEC_BATCHER_WORKERS=\$w $OUT/bench_batcher 64 32 0 96 300 && HBEC_BATCHER_WORKERS=\$w $OUT/bench_batcher 16 128 1 96 300 || exit 1; done" ;;
    soak)
      gcc -O2 -std=c11 -pthread -Iinclude scripts/soak.c -Lhummingbird_amd -lhbec -Wl,-rpath,$ROOT/hummingbird_amd -o $OUT/soak && step soak 400 sh -c "$OUT/soak 8 20 && $OUT/soak 48 60 && $OUT/soak 128 40" ;;
    md5tests) step md5tests 600 python -m pytest tests/test_gpu_md5.py -q -x -p no:cacheprovider ;;
    md5) step md5 600 python scripts/bench_md5.py ;;
    md5sweep) step md5sweep 900 bash scripts/md5_sweep.sh ;;
    tuneplan) step tuneplan 1000 bash scripts/tune_plan.sh ;;
    md5prof)
      mkdir -p "$OUT/md5prof"
      (cd /tmp && step md5prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/md5prof" -o run -- python3 "$ROOT/scripts/bench_md5.py") || exit $?
      ;;
    seq) step seq 600 python scripts/tune.py seq ;;
    xorsweep) step xorsweep 600 python scripts/tune.py xorsweep ;;
    copysweep) step copysweep 600 python scripts/tune.py copysweep ;;
    layout) step layout 600 python scripts/tune.py layout ;;
    probe) step probe 600 python scripts/tune.py probe ;;
    tune) step tune 900 python scripts/tune.py run ${TUNE_ARGS:-} ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
