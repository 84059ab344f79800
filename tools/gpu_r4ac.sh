# Round-4 closing measurements on the final build (second session): every -m gpu test, smoke,
# the driver's bench command, then tools/gpu_r4_final.sh (bench lines, kernel traces, C2 PMC passes)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r4ac.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r4ac.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && { grep -E "FAILED|ERROR" gpurun_out/pytest_r4ac.log | head; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4ac.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_r4ac.log; exit 1; }
tail -1 gpurun_out/smoke_r4ac.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r4ac_driver.json 2> gpurun_out/bench_r4ac_driver.err || { echo driver bench failed; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4ac_driver.json'));print('driver form', d['value'], d['runs'])"
bash tools/gpu_r4_final.sh r04g
