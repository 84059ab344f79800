#!/bin/bash
# A/B on the GPU box: the particle GPU tests with the in-tree library, then bench lines of the
# in-tree library and of each experiment library given.   tools/gpu_ab.sh CONFIG TESTS lib.so ...
set -o pipefail
cfg=$1; shift; tests=$1; shift
mkdir -p gpurun_out
if [ -n "$tests" ]; then
  timeout -k 10 600 python3 -u -m pytest $tests -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_ab.log; grep -E "FAILED|ERROR" gpurun_out/pytest_ab.log | head
  [ $rc -ne 0 ] && exit $rc
fi
case $cfg in
  halfcheetah) args="--steps 2000 --warmup 100";;
  humanoid) args="--config humanoid --steps 600 --warmup 50";;
  particles) args="--config particles --steps 20 --warmup 3";;
esac
BENCH_ARGS="$args" bash tools/run_libs.sh td3_amd/libtd3hip.so "$@"
