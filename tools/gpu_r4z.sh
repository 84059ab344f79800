# Round-4 closing check at HEAD: every -m gpu test, smoke(), and the driver's bench command
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
set -o pipefail
bash tools/gpu_round.sh r4z || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4z.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_r4z.log; exit 1; }
tail -1 gpurun_out/smoke_r4z.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r4z_driver.json 2> gpurun_out/bench_r4z_driver.err || { echo driver bench failed; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4z_driver.json'));print('driver form', d['value'], d['runs'], d['roofline']['frac'], d['cpu_baseline']['value'])"
