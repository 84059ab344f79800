# round-4 closing measurements on the final build: every config's bench line, rocprofv3 kernel stats
# of the C2 and Humanoid bench commands, the C2 PMC passes (FETCH / WRITE) for pmc_traffic.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
tag=${1:-r04f}
for c in halfcheetah pendulum humanoid particles; do
  extra=""; [ $c = particles ] && extra="--steps 60 --warmup 10"
  timeout -k 10 400 python3 bench.py --config $c $extra > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_${tag}_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${tag}_$c.json'));print('$c',d['value'],d['runs'],d['roofline']['kernel'],d['roofline']['frac'],d['cpu_baseline']['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o run -- python3 bench.py --steps 300 --warmup 30 --runs 1 --no-cpu-baseline > gpurun_out/prof_${tag}.log 2>&1 || { echo trace failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profh_${tag} -o run -- python3 bench.py --config humanoid --steps 100 --warmup 20 --runs 1 --no-cpu-baseline > gpurun_out/profh_${tag}.log 2>&1 || { echo htrace failed; exit 1; }
echo traces ok
C="--steps 20 --warmup 5 --runs 1 --no-cpu-baseline --no-roofline"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${tag}_cf -o run -- python3 bench.py $C > gpurun_out/pmc_${tag}_cf.log 2>&1 || { echo "pmc cf failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${tag}_cw -o run -- python3 bench.py $C > gpurun_out/pmc_${tag}_cw.log 2>&1 || { echo "pmc cw failed"; exit 1; }
echo pmc ok
