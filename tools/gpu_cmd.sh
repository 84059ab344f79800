set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_w4.py tests/test_gpu_data_parallel.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pw4.log 2>&1; rc=$?; echo "w4+dp tests rc=$rc"; tail -3 gpurun_out/pw4.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
TD3_DP_SHARD=2 TD3_W4=$v timeout -k 10 200 python3 bench.py --dp-self --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/b_w4ds_$v.json 2>/dev/null; echo "dp-self shard w4=$v rc=$?"; python3 -c "
import json;d=json.loads(open('gpurun_out/b_w4ds_$v.json').read().strip().splitlines()[-1]);print(d['value'],d.get('runs'))"
done
