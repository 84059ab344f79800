# split-K: two 64-row steps per barrier (TD3_DWSK_DEPTH=5) against one; bitwise test over every walk
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "split_dw_walks" --timeout 150 --timeout-method thread > gpurun_out/pytest_r4l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4l.log; [ $rc -eq 0 ] || exit 1
for cfg in "0 5" "0 2" "0 5"; do
  set -- $cfg
  TD3_DWSK_ORDER=$1 TD3_DWSK_DEPTH=$2 timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_l_o$1_d$2.json 2> gpurun_out/hum_l_o$1_d$2.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_l_o$1_d$2.json'));print('order $1 depth $2',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
TD3_DWSK_DEPTH=5 timeout -k 10 300 python3 bench.py --config particles --steps 30 --warmup 5 --runs 3 --no-cpu-baseline > gpurun_out/part_d5.json 2> gpurun_out/part_d5.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/part_d5.json'));print('particles depth 5',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
