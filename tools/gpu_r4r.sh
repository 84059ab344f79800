# td3_sync = hipStreamSynchronize: GPU suite (data-parallel tests last, non-fatal), the driver form x3,
# the default C2 line
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --ignore=tests/test_gpu_data_parallel.py > gpurun_out/pytest_r4r.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4r.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r4r_driver$i.json 2> gpurun_out/bench_r4r_driver$i.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_r4r_driver$i.json').read().strip().splitlines()[-1]);print('driver form',d['value'],d['runs'])"
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_r4r.json 2> gpurun_out/bench_r4r.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4r.json'));print('C2 default',d['value'],d['runs'],d['roofline']['avg_launch_us'],d['cpu_baseline']['value'])"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_data_parallel.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r4r_dp.log 2>&1
echo "dp pytest rc=$?"; grep -E "passed|failed|AssertionError|assert " gpurun_out/pytest_r4r_dp.log | head -20
