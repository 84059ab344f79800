# split-K dW LDS ring depth: parity (bitwise across walks, gradients through Adam at B=1024), then
# Humanoid A/B over TD3_DWSK_DEPTH (stage times), then the short-run anatomy probes
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gradients.py -m gpu -q -k "split_dw_walks or large_batch or hum_b1024 or hum_layer" --timeout 120 --timeout-method thread > gpurun_out/pytest_r4e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4e.log; [ $rc -eq 0 ] || exit 1
for d in 2 3 4; do
  TD3_DWSK_DEPTH=$d timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_depth$d.json 2> gpurun_out/hum_depth$d.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_depth$d.json'));print('depth $d',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
bash tools/gpu_r4d.sh
