#!/bin/bash
# GPU-box check: parity tests, the C2 bench line and the acting-loop bench.  Usage: tools/gpu_check2.sh TAG
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_$tag.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$tag.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
timeout -k 10 300 python3 bench_loop.py > gpurun_out/loop_$tag.json 2> gpurun_out/loop_$tag.err || { tail -20 gpurun_out/loop_$tag.err; exit 1; }
python3 - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/bench_{t}.json", f"gpurun_out/loop_{t}.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d.get("roofline", {}).get("frac"), d.get("serial_value"))
PY
