#!/bin/bash
# Bench several builds of libtd3hip (GPU box).  Usage: [BENCH_ARGS="--config particles"] tools/run_libs.sh a.so b.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  tag=$(basename $lib .so)
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/lib_$tag.json 2> gpurun_out/lib_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/lib_$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lib_$tag.json').read().strip().splitlines()[-1])
print('$tag', d['value'], {k:v for k,v in d['stage_us'].items() if k.startswith('1:')})"
done
