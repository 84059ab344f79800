#!/bin/bash
# Round profile set (GPU box): C2 bench + rocprofv3 kernel stats + PMC traffic passes
# (tools/profile_round.sh), then the Humanoid / particles bench lines and the acting loop.
#   tools/profile_all.sh r02   -> gpurun_out/{bench,prof,pmcf,pmcw}_r02*, gpurun_out/*_r02.json
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
bash tools/profile_round.sh $tag || exit 1
timeout -k 10 300 python3 bench.py --config humanoid > gpurun_out/bench_humanoid_$tag.json 2> gpurun_out/bench_humanoid_$tag.err || { echo humanoid failed; tail gpurun_out/bench_humanoid_$tag.err; exit 1; }
echo "humanoid ok: $(cut -c1-160 gpurun_out/bench_humanoid_$tag.json)"
timeout -k 10 400 python3 bench.py --config particles --steps 300 --warmup 20 > gpurun_out/bench_particles_$tag.json 2> gpurun_out/bench_particles_$tag.err || { echo particles failed; tail gpurun_out/bench_particles_$tag.err; exit 1; }
echo "particles ok: $(cut -c1-160 gpurun_out/bench_particles_$tag.json)"
timeout -k 10 300 python3 bench_loop.py > gpurun_out/bench_loop_$tag.json 2> gpurun_out/bench_loop_$tag.err || { echo loop failed; tail gpurun_out/bench_loop_$tag.err; exit 1; }
echo "loop ok: $(cut -c1-160 gpurun_out/bench_loop_$tag.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_humanoid_$tag -o run -- python3 bench.py --config humanoid --steps 300 --warmup 30 --no-cpu-baseline --no-roofline > gpurun_out/prof_humanoid_$tag.log 2>&1 || { echo humanoid trace failed; tail gpurun_out/prof_humanoid_$tag.log; exit 1; }
echo "humanoid trace ok"
