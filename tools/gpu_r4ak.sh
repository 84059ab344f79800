# C2: 16-column GEMM workgroups for stages of up to 208 / 256 32-column workgroups (TD3_WN0_MAX)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
for L in tools/exp/libtd3hip_wn0m208.so tools/exp/libtd3hip_wn0m256.so; do
  TD3_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4ak.log 2>&1 || { echo "pytest failed $L"; tail -20 gpurun_out/pytest_r4ak.log; exit 1; }
  tail -1 gpurun_out/pytest_r4ak.log
done
for lib in td3_amd/libtd3hip.so tools/exp/libtd3hip_wn0m208.so tools/exp/libtd3hip_wn0m256.so td3_amd/libtd3hip.so tools/exp/libtd3hip_wn0m208.so tools/exp/libtd3hip_wn0m256.so; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4ak.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4ak.json'));s=d['stage_us'];print('$lib', d['value'], s)"
done
