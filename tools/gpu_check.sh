#!/bin/bash
# GPU-box check: parity tests, then a bench line.  Usage: tools/gpu_check.sh TAG [bench args]
set -o pipefail
tag=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$tag.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$tag.err; exit $rc; }
python3 - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(d["value"], d.get("roofline"))
print(d.get("stage_us"))
print(d.get("cpu_baseline"))
PY
