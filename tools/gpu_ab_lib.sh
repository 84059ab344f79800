#!/bin/bash
# Parity subset, then a bench A/B, for experiment libraries (GPU box).  tools/gpu_ab_lib.sh CONFIG lib.so ...
set -o pipefail
cfg=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  tag=$(basename $lib .so)
  TD3_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
  rc=$?; echo "$tag pytest rc=$rc: $(tail -1 gpurun_out/pytest_$tag.log)"
  [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_ab.sh $cfg "" "$@"
