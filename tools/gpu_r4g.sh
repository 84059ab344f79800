# Humanoid C_dw / A_dw per-workgroup timeline (balance of the split-K partition), and a kernel trace of
# the bucketed data-parallel schedule on a one-rank communicator (where its extra time goes)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TD3_LIB=tools/exp/libtd3hip_tl.so TL_SHAPE=376,17,1024 TL_DUMP=gpurun_out/tl_hum timeout -k 10 200 python3 tools/tl_probe.py > gpurun_out/tl_hum.log 2>&1 || { tail -5 gpurun_out/tl_hum.log; exit 1; }
grep -E "C_dw|A_dw|==" gpurun_out/tl_hum.log
TD3_DP_BUCKETS=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_bk -o run -- python3 bench.py --config humanoid --dp-self --steps 30 --warmup 10 --runs 1 --no-cpu-baseline --no-roofline > gpurun_out/trace_bk.log 2>&1 || { tail -5 gpurun_out/trace_bk.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_nb -o run -- python3 bench.py --config humanoid --dp-self --steps 30 --warmup 10 --runs 1 --no-cpu-baseline --no-roofline > gpurun_out/trace_nb.log 2>&1 || { tail -5 gpurun_out/trace_nb.log; exit 1; }
echo traces ok
