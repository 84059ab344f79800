# Layer-0 LayerNorm (kProL0 / kProL0G) with its rows' LDS reads batched: parity subset, C2 / Humanoid A/B
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
L=tools/exp/libtd3hip_l0ln.so
TD3_LIB=$L timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py tests/test_gpu_gradients.py tests/test_gpu_data_parallel.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r4ah.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_r4ah.log; exit 1; }
tail -1 gpurun_out/pytest_r4ah.log
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4ah.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ah.json'));s=d['stage_us'];print('$lib', d['value'], {k:v for k,v in s.items() if k[2:] in ('F_fwd01','CB_bwd2+TF_fwd01','AF_fwd01')})"
done
for lib in td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --config humanoid --steps 600 --warmup 50 --runs 3 --no-cpu-baseline > gpurun_out/r4ah_h.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ah_h.json'));s=d['stage_us'];print('humanoid $lib', d['value'], {k:v for k,v in s.items() if k[2:] in ('heads','critic_loss')})"
done
