set -o pipefail
F=gpurun_out/g1
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/pytest.log 2>&1
rc=$?; tail -2 $F/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $F/prof_h -o run -- python3 bench.py \
  --config humanoid --steps 300 --warmup 30 --no-cpu-baseline --no-roofline > $F/prof_h.log 2>&1; echo "prof rc=$?"
timeout -k 10 300 python3 bench.py --config humanoid --steps 600 --warmup 50 > $F/bench_h.json 2> $F/bench_h.err; echo "bench rc=$?"
