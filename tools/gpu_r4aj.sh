# C2: the target twin's fused layer 0-1 (TF_fwd01, in the dual launch with CB_bwd2) at 64 output
# columns (TD3_WN2_MIN=200: 104 workgroups instead of 208) against the product
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
L=tools/exp/libtd3hip_tfwn2.so
TD3_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4aj.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_r4aj.log; exit 1; }
tail -1 gpurun_out/pytest_r4aj.log
for lib in td3_amd/libtd3hip.so $L td3_amd/libtd3hip.so $L; do
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4aj.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4aj.json'));s=d['stage_us'];print('$lib', d['value'], {k:v for k,v in s.items() if 'CB_bwd2' in k})"
done
