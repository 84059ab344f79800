# DP tests (the critic against the DP-form oracle), then the round-4 closing measurements
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_data_parallel.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r4u_dp.log 2>&1
echo "dp pytest rc=$?"; grep -E "passed|failed|Error" gpurun_out/pytest_r4u_dp.log | head -10
bash tools/gpu_r4_final.sh r04f
