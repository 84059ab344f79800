# In-kernel phase timelines of the HalfCheetah B=256 GEMM stages (TD3_TL build)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
TD3_LIB=tools/exp/libtd3hip_tl.so timeout -k 10 200 python3 -u tools/tl_probe.py > gpurun_out/r4y_tl_hc.txt 2>&1 || { echo "tl hc failed"; tail gpurun_out/r4y_tl_hc.txt; exit 1; }
grep -v "clock(mfma" gpurun_out/r4y_tl_hc.txt | head -80
