# In-kernel phase timelines of the Humanoid B=1024 and HalfCheetah B=256 GEMM stages (TD3_TL build)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
TL_SHAPE=376,17,1024 TD3_LIB=tools/exp/libtd3hip_tl.so timeout -k 10 200 python3 -u tools/tl_probe.py > gpurun_out/r4y_tl_hum.txt 2>&1 || { echo "tl hum failed"; tail gpurun_out/r4y_tl_hum.txt; exit 1; }
cat gpurun_out/r4y_tl_hum.txt | tail -40
