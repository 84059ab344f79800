# Row kernels with their output addresses / noise parameters held in VGPRs (no scalar kernel-argument
# reloads in the waves' tails): parity subset, C2 / Humanoid A/B
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
L=tools/exp/libtd3hip_vpin.so
TD3_LIB=$L timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py tests/test_gpu_gradients.py tests/test_gpu_data_parallel.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r4ag.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_r4ag.log; exit 1; }
tail -1 gpurun_out/pytest_r4ag.log
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4ag.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ag.json'));s=d['stage_us'];print('$lib', d['value'], {k:v for k,v in s.items() if k[2:] in ('heads','critic_loss','actor_head_bwd','AB_lnbwd0')})"
done
for lib in td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --config humanoid --steps 600 --warmup 50 --runs 3 --no-cpu-baseline > gpurun_out/r4ag_h.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ag_h.json'));s=d['stage_us'];print('humanoid $lib', d['value'], {k:v for k,v in s.items() if k[2:] in ('heads','critic_loss')})"
done
