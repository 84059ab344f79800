# dw_kernel k-tile pairs (TD3_DW_KP): bitwise test, then C2 A/B (long runs and the driver form)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "kpair or teacher_forced or graph_equals" > gpurun_out/pytest_r4v.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_r4v.log; exit 1; }
tail -2 gpurun_out/pytest_r4v.log
for kp in 1 2 1 2; do
  TD3_DW_KP=$kp timeout -k 10 240 python3 -u bench.py --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline > gpurun_out/r4v_kp${kp}.json 2> gpurun_out/r4v_kp${kp}.err || { echo "bench kp=$kp failed"; tail gpurun_out/r4v_kp${kp}.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/r4v_kp$kp.json'));s=d['stage_us'];print('kp=$kp', d['value'], d['runs'], 'C_dw', s['0:C_dw'], s['1:C_dw'], 'A_dw', s['1:A_dw'])"
done
for kp in 1 2; do
  TD3_DW_KP=$kp timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/r4v_drv_kp${kp}.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4v_drv_kp$kp.json'));print('driver form kp=$kp', d['value'], d['runs'])"
done
