# F_fwd01: branch-free Philox draws + record addresses formed before them (no scalar reloads
# between the draws and the record loads): parity subset + C2 A/B (replay and whole step)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
L=tools/exp/libtd3hip_philox.so
TD3_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4ad.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_r4ad.log; exit 1; }
tail -1 gpurun_out/pytest_r4ad.log
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4ad.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ad.json'));r=d['roofline'];s=d['stage_us'];print('$lib', d['value'], 'F_fwd01 replay', s['0:F_fwd01'], s['1:F_fwd01'], 'in-step', r['in_step_launch_us'])"
done
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/r4ad_drv.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ad_drv.json'));print('driver form $lib', d['value'], d['runs'])"
done
