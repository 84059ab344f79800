# per-workgroup timelines of the pipelined split-K walk (Humanoid C_dw / A_dw) for the cost fit
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TD3_DWSK_ORDER=2 TD3_LIB=tools/exp/libtd3hip_tl.so TL_SHAPE=376,17,1024 TL_DUMP=gpurun_out/tl_hum2 timeout -k 10 200 python3 tools/tl_probe.py > gpurun_out/tl_hum2.log 2>&1 || { tail -5 gpurun_out/tl_hum2.log; exit 1; }
grep -E "C_dw|A_dw" -A5 gpurun_out/tl_hum2.log | grep -E "C_dw|A_dw|end p10"
