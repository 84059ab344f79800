# Unconditional first streamed loads in the fused layer-0 stages only: parity subset, C2 / Humanoid A/B
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
L=tools/exp/libtd3hip_ustream3.so
TD3_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_gradients.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4ab.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_r4ab.log; exit 1; }
tail -1 gpurun_out/pytest_r4ab.log
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ab.json'));r=d['roofline'];print('$lib', d['value'], 'F_fwd01 replay', r['avg_launch_us'], 'in-step', r['in_step_launch_us'])"
done
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/r4ab_drv.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ab_drv.json'));print('driver form $lib', d['value'], d['runs'])"
done
for lib in td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --config humanoid --steps 600 --warmup 50 --runs 3 --no-cpu-baseline --no-roofline > gpurun_out/r4ab_h.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ab_h.json'));print('humanoid $lib', d['value'])"
done
