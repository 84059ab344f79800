# C2: odd-step F_fwd01 / even F_fwd2 at 32 output columns (TD3_WN2_MIN=400) against the product
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
bash tools/gpu_ab_lib.sh halfcheetah tools/exp/libtd3hip_wn2m400.so || exit 1
BENCH_ARGS="--steps 2000 --warmup 100" bash tools/run_libs.sh td3_amd/libtd3hip.so tools/exp/libtd3hip_wn2m400.so
