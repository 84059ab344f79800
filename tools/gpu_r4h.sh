# pipelined split-K walk (TD3_DWSK_ORDER=2) vs tile-major: bitwise test, gradients, Humanoid + particles A/B
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gradients.py -m gpu -q -k "split_dw_walks or hum_b1024" --timeout 150 --timeout-method thread > gpurun_out/pytest_r4h.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4h.log; [ $rc -eq 0 ] || exit 1
for o in 0 2; do
  TD3_DWSK_ORDER=$o timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_ord$o.json 2> gpurun_out/hum_ord$o.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_ord$o.json'));print('humanoid order $o',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
for o in 0 2; do
  TD3_DWSK_ORDER=$o timeout -k 10 300 python3 bench.py --config particles --steps 30 --warmup 5 --runs 3 --no-cpu-baseline > gpurun_out/part_ord$o.json 2> gpurun_out/part_ord$o.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/part_ord$o.json'));print('particles order $o',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_data_parallel.py -m gpu -q -k "overlapped or c5 or local_replicas" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4h_dp.log 2>&1
rc=$?; echo "dp pytest rc=$rc"; tail -3 gpurun_out/pytest_r4h_dp.log; [ $rc -eq 0 ] || exit 1
for bk in 0 2; do
  TD3_DP_BUCKETS=$bk timeout -k 10 200 python3 bench.py --config humanoid --dp-self --steps 300 --warmup 30 --runs 3 --no-cpu-baseline --no-roofline > gpurun_out/hdp_bk$bk.json 2> gpurun_out/hdp_bk$bk.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/hdp_bk$bk.json').read().strip().splitlines()[-1]);print('dp-self humanoid buckets $bk',d['value'],d['runs'])"
done
