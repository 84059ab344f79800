# A/B of the split-K dW walk on Humanoid (stage times), the short-run probe of the C2 driver form
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "split_dw_walk or large_batch" --timeout 120 --timeout-method thread > gpurun_out/pytest_r4c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r4c.log; [ $rc -eq 0 ] || exit 1
for o in 1 0; do
  TD3_DWSK_ORDER=$o timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_order$o.json 2> gpurun_out/hum_order$o.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_order$o.json'));print('order $o',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
timeout -k 10 120 python3 tools/short_probe.py > gpurun_out/short_probe.log 2>&1 || exit 1
cat gpurun_out/short_probe.log | grep run
