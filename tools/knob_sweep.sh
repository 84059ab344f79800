#!/bin/bash
# Humanoid bench under planner env knobs (GPU box).  tools/knob_sweep.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 200 python3 bench.py ${KNOB_ARGS:---config humanoid --steps 600 --warmup 50} --no-cpu-baseline > gpurun_out/knob_$i.json 2> gpurun_out/knob_$i.err || { echo "[$kv] failed"; tail -3 gpurun_out/knob_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/knob_$i.json').read().strip().splitlines()[-1])
print('[$kv]', d['value'], {k:v for k,v in d['stage_us'].items() if True})"
done
