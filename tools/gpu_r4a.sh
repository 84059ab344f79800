# round-4 GPU check: gradient parity, full GPU suite, short-run kernel trace, Humanoid dW order A/B,
# the default bench line
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gradients.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_grad.log 2>&1
echo "grad rc=$?"; tail -8 gpurun_out/pytest_grad.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4a.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_short -o run -- python3 bench.py --steps 20 --warmup 5 --runs 10 --no-cpu-baseline --no-roofline > gpurun_out/kt_short.log 2>&1 || exit 1
for o in 1 0; do
  TD3_DWSK_ORDER=$o timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_order$o.json 2> gpurun_out/hum_order$o.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_order$o.json'));print('order $o',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4a.json'));print('C2',d['value'],d['runs'])"
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-roofline --no-cpu-baseline > gpurun_out/bench_r4a_driver.json 2>&1 || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4a_driver.json'));print('C2 driver-form',d['value'],d['runs'])"
