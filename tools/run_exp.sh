#!/bin/bash
# Bench each experiment variant (GPU box).  Usage: tools/run_exp.sh 1 2 3
set -o pipefail
mkdir -p gpurun_out
for e in "$@"; do
  TD3_LIB=tools/exp/libtd3hip_exp$e.so timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/exp$e.json 2> gpurun_out/exp$e.err || { echo "exp$e failed"; tail -5 gpurun_out/exp$e.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/exp$e.json').read().strip().splitlines()[-1])
print('exp$e', d['value'], {k:v for k,v in d['stage_us'].items() if k.startswith('1:')})"
done
