#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_plan.py tests/test_gpu_bitplane.py tests/test_gpu_unaligned.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_b1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_b1_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > gpurun_out/r5_bench1.json 2> gpurun_out/r5_bench1.err || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r5_bench1.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["roofline"]["frac"])
o = d["odd_objects"]
print("odd 4+2", {k: o[k]["frac"] for k in ("encode", "reconstruct", "verify")})
for s, v in o["shapes"].items():
    print("odd", s, {k: v[k]["frac"] for k in ("encode", "reconstruct", "verify")})
print("random", json.dumps(d["random_objects"])[:600])
print("config4", d["config4"].get("frac"), "small", {k: v for k, v in d["small_objects"].items() if k != "workload"} if isinstance(d["small_objects"], dict) else None)
PY
