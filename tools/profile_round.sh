#!/bin/bash
# Round profile (GPU box): bench line + rocprofv3 kernel stats + PMC HBM-traffic passes.
#   tools/profile_round.sh r01      -> gpurun_out/prof_r01*/ ; copy into profiles/ afterwards
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
B="bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-roofline"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo bench failed; tail gpurun_out/bench_$tag.err; exit 1; }
echo "bench ok: $(cut -c1-200 gpurun_out/bench_$tag.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 $B > gpurun_out/prof_$tag.log 2>&1 || { echo trace failed; tail gpurun_out/prof_$tag.log; exit 1; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$tag -o run -- python3 $B > gpurun_out/pmcf_$tag.log 2>&1 || { echo pmc fetch failed; tail gpurun_out/pmcf_$tag.log; exit 1; }
echo pmc fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$tag -o run -- python3 $B > gpurun_out/pmcw_$tag.log 2>&1 || { echo pmc write failed; tail gpurun_out/pmcw_$tag.log; exit 1; }
echo pmc write ok
find gpurun_out/prof_$tag gpurun_out/pmcf_$tag gpurun_out/pmcw_$tag -name "*.csv" | head -20
