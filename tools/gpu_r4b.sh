# round-4 profiles: rocprofv3 kernel stats of the default bench command, the Pendulum (C1) line with its
# cpu_baseline, Humanoid / particles lines, and the Humanoid C_dw PMC passes (FETCH / WRITE / L2 hit)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
tag=${1:-r04}
timeout -k 10 300 python3 bench.py --config pendulum > gpurun_out/bench_${tag}_pendulum.json 2> gpurun_out/bench_${tag}_pendulum.err || { echo pendulum failed; tail -5 gpurun_out/bench_${tag}_pendulum.err; exit 1; }
echo "pendulum ok: $(cut -c1-160 gpurun_out/bench_${tag}_pendulum.json)"
timeout -k 10 300 python3 bench.py --config humanoid > gpurun_out/bench_${tag}_humanoid.json 2> gpurun_out/bench_${tag}_humanoid.err || { echo humanoid failed; exit 1; }
echo "humanoid ok: $(cut -c1-160 gpurun_out/bench_${tag}_humanoid.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o run -- python3 bench.py --steps 300 --warmup 30 --runs 1 --no-cpu-baseline > gpurun_out/prof_${tag}.log 2>&1 || { echo trace failed; tail -5 gpurun_out/prof_${tag}.log; exit 1; }
echo "trace ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profh_${tag} -o run -- python3 bench.py --config humanoid --steps 100 --warmup 20 --runs 1 --no-cpu-baseline > gpurun_out/profh_${tag}.log 2>&1 || { echo htrace failed; exit 1; }
echo "htrace ok"
H="--config humanoid --steps 20 --warmup 5 --runs 1 --no-cpu-baseline --no-roofline"
for pass in "hf FETCH_SIZE" "hw WRITE_SIZE" "hl TCC_HIT_sum TCC_MISS_sum"; do
  set -- $pass; name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc $@ --output-format csv -d gpurun_out/pmc_${tag}_$name -o run -- python3 bench.py $H > gpurun_out/pmc_${tag}_$name.log 2>&1 || { echo "pmc $name failed"; tail -3 gpurun_out/pmc_${tag}_$name.log; exit 1; }
  echo "pmc $name ok"
done
timeout -k 10 200 python3 bench.py --dp-self --no-cpu-baseline --runs 3 > gpurun_out/bench_${tag}_dpself.json 2> gpurun_out/bench_${tag}_dpself.err || { echo dpself failed; tail -5 gpurun_out/bench_${tag}_dpself.err; exit 1; }
echo "dpself ok: $(cut -c1-160 gpurun_out/bench_${tag}_dpself.json)"
timeout -k 10 200 python3 bench.py --config humanoid --dp-self --no-cpu-baseline --runs 3 > gpurun_out/bench_${tag}_hdpself.json 2> gpurun_out/bench_${tag}_hdpself.err || { echo hdpself failed; exit 1; }
echo "hdpself ok: $(cut -c1-160 gpurun_out/bench_${tag}_hdpself.json)"
timeout -k 10 200 env TD3_DP_BUCKETS=2 python3 bench.py --config humanoid --dp-self --no-cpu-baseline --runs 3 > gpurun_out/bench_${tag}_hdpself_b.json 2> gpurun_out/bench_${tag}_hdpself_b.err || { echo hdpself_b failed; exit 1; }
echo "hdpself buckets ok: $(cut -c1-160 gpurun_out/bench_${tag}_hdpself_b.json)"
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${tag}_driver$i.json 2> gpurun_out/bench_${tag}_driver$i.err || { echo driver failed; exit 1; }
  echo "driver form $i: $(cut -c1-200 gpurun_out/bench_${tag}_driver$i.json)"
done
