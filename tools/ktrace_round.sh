#!/bin/bash
# rocprofv3 kernel stats of the Humanoid and particle bench commands + the acting-loop bench (GPU box).
#   tools/ktrace_round.sh r03   -> gpurun_out/ktrace_r03_{humanoid,particles}/, gpurun_out/bench_loop_r03.json
set -o pipefail
tag=${1:-r03}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for c in humanoid particles; do
  case $c in
    humanoid) args="--config humanoid --steps 300 --warmup 30";;
    particles) args="--config particles --steps 10 --warmup 2";;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace_${tag}_$c -o run -- \
    python3 bench.py $args --no-cpu-baseline --no-roofline > gpurun_out/ktrace_${tag}_$c.log 2>&1 \
    || { echo "trace $c failed"; tail gpurun_out/ktrace_${tag}_$c.log; exit 1; }
  echo "trace $c ok"
done
timeout -k 10 300 python3 bench_loop.py > gpurun_out/bench_loop_$tag.json 2> gpurun_out/bench_loop_$tag.err \
  || { echo "loop bench failed"; tail gpurun_out/bench_loop_$tag.err; exit 1; }
tail -1 gpurun_out/bench_loop_$tag.json | cut -c1-400
find gpurun_out/ktrace_${tag}_* -name "*stats*.csv"
