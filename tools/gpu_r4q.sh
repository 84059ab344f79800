# LDS-staged wide head backward (bitwise test + Humanoid line); td3_sync modes in the short-run regime
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gradients.py tests/test_gpu_fullsize.py -m gpu -q -k "wide_head or hum or c3" --timeout 200 --timeout-method thread > gpurun_out/pytest_r4q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4q.log; [ $rc -eq 0 ] || exit 1
for f in 1 0; do
  TD3_HEAD_LDS=$f timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_hl$f.json 2> gpurun_out/hum_hl$f.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_hl$f.json'));print('head lds $f',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'head' in k})"
done
for m in 0 1 2; do
  TD3_SYNC_MODE=$m SP_MODE=syncs timeout -k 10 200 python3 tools/short_probe.py > gpurun_out/sp_syncs_m$m.log 2>&1 || exit 1
  grep "td3_sync + torch" gpurun_out/sp_syncs_m$m.log | sed "s/^/mode $m: /"
  TD3_SYNC_MODE=$m SP_MODE=plain timeout -k 10 200 python3 tools/short_probe.py > gpurun_out/sp_plain_m$m.log 2>&1 || exit 1
  grep "run [0-7]" gpurun_out/sp_plain_m$m.log | sed "s/^/mode $m: /" | cut -c1-140
done
for m in 0 1; do for i in 1 2; do
  TD3_SYNC_MODE=$m timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/c2_sync_m${m}_$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c2_sync_m${m}_$i.json'));print('driver form sync mode $m',d['value'],d['runs'])"
done; done
