# split wide policy head: bitwise test, Humanoid parity subset, A/B of the heads stage
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gradients.py tests/test_gpu_fullsize.py -m gpu -q -k "split_policy or hum or c3 or select" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4s.log; [ $rc -eq 0 ] || exit 1
for f in 1 0; do
  TD3_HEAD_SPLIT=$f timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_hs$f.json 2> gpurun_out/hum_hs$f.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_hs$f.json'));print('head split $f',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'head' in k})"
done
