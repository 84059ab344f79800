# wide policy heads loaded per block: full GPU suite, Humanoid line
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r4o.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4o.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --config humanoid --runs 3 --no-cpu-baseline > gpurun_out/bench_r4o_humanoid.json 2> gpurun_out/bench_r4o_humanoid.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_r4o_humanoid.json'));print('humanoid',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'head' in k})"
for kn in "224 288" "400 640" "340 640"; do
  set -- $kn
  TD3_WN4_MIN=$1 TD3_WN2_MAXB=$2 timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_wn_$1_$2.json 2> gpurun_out/hum_wn_$1_$2.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_wn_$1_$2.json'));print('wn4_min $1 wn2_maxb $2',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'fwd' in k or 'bwd' in k})"
done
