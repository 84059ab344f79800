# Unconditional (clamped) streamed weight loads in the GEMM stages: parity subset, C2 and Humanoid A/B
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
bash tools/gpu_ab_lib.sh halfcheetah tools/exp/libtd3hip_ustream2.so || exit 1
BENCH_ARGS="--steps 2000 --warmup 100" bash tools/run_libs.sh td3_amd/libtd3hip.so tools/exp/libtd3hip_ustream2.so || exit 1
BENCH_ARGS="--config humanoid --steps 600 --warmup 50" bash tools/run_libs.sh td3_amd/libtd3hip.so tools/exp/libtd3hip_ustream2.so td3_amd/libtd3hip.so tools/exp/libtd3hip_ustream2.so || exit 1
for lib in td3_amd/libtd3hip.so tools/exp/libtd3hip_ustream2.so; do
  TD3_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/r4aa_drv.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4aa_drv.json'));print('driver form $lib', d['value'], d['runs'])"
done
