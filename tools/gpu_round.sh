#!/bin/bash
# GPU-box round check: every -m gpu test (all failures listed), then bench lines per config.
# Stops at the first step that ends in a time limit / abort / segfault (124 137 134 139) -- a
# failing assert (pytest rc 1) does not stop the benches.
#   tools/gpu_round.sh TAG [configs...]      (configs: halfcheetah humanoid particles; default hc)
set -o pipefail
tag=${1:-run}; shift
cfgs=${*:-halfcheetah}
mkdir -p gpurun_out
fatal() { case $1 in 124|137|134|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_$tag.log; echo "pytest rc=$rc"
grep -E "FAILED|ERROR" gpurun_out/pytest_$tag.log | head -20
fatal $rc && exit $rc
# a GPU fault leaves the context unusable: stop before the benches run into it again
if grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault" gpurun_out/pytest_$tag.log; then
  echo "GPU fault in the tests: no benches"; exit 3
fi
for c in $cfgs; do
  case $c in
    halfcheetah) args="--steps 2000 --warmup 100";;
    humanoid) args="--config humanoid --steps 600 --warmup 50";;
    particles) args="--config particles --steps 20 --warmup 3";;
  esac
  timeout -k 10 400 python3 bench.py $args > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err
  rc=$?; echo "bench $c rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${tag}_$c.err; fatal $rc && exit $rc; continue; }
  python3 - "gpurun_out/bench_${tag}_$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(d["value"], d["ms_per_step"], "dom", r.get("kernel"), r.get("frac"), "step_frac", r.get("step_frac"))
print("gather", d.get("gather"))
print("stages", d.get("stage_us"))
print("cpu", d.get("cpu_baseline"))
PY
done
exit 0
