# round-4 GPU check: short-run kernel trace, then the gradient parity tests, then the full GPU suite
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_short -o run -- python3 bench.py --steps 20 --warmup 5 --runs 10 --no-cpu-baseline --no-roofline > gpurun_out/kt_short.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gradients.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_grad.log 2>&1
echo "grad rc=$?"; tail -8 gpurun_out/pytest_grad.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r4a.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/pytest_r4a.log
