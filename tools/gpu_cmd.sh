set -o pipefail
F=gpurun_out/g4
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_combine.py -x -v --timeout 120 --timeout-method thread > $F/comb.log 2>&1
rc=$?; tail -6 $F/comb.log; echo "comb rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/pytest.log 2>&1
rc=$?; tail -2 $F/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $F/prof_h -o run -- python3 bench.py \
  --config humanoid --steps 300 --warmup 30 --no-cpu-baseline --no-roofline > $F/prof_h.log 2>&1; echo "prof rc=$?"
for i in 1 2; do
TD3_COMB_FAST=0 timeout -k 10 300 python3 bench.py --config humanoid --steps 600 --warmup 50 --no-cpu-baseline --no-roofline > $F/bench_h0_$i.json 2> $F/bench_h0_$i.err; echo "bench0 rc=$?"
timeout -k 10 300 python3 bench.py --config humanoid --steps 600 --warmup 50 --no-cpu-baseline --no-roofline > $F/bench_h1_$i.json 2> $F/bench_h1_$i.err; echo "bench1 rc=$?"
done
for f in $F/bench_h*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'])"; done
grep -E "combine|row_kernel<3" $F/prof_h/run_kernel_stats.csv | cut -c1-120
