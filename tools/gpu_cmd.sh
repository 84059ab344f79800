set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pall.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pall.log; grep -E "FAILED|ERROR" gpurun_out/pall.log | head -20
case $rc in 124|137|134|139) exit $rc;; esac
grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault" gpurun_out/pall.log && { echo "GPU fault"; exit 3; }
for v in 0 1 0 1; do
TD3_W4=$v timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/b_w4r_$v.json 2>/dev/null; echo "bench w4=$v rc=$?"; python3 -c "
import json;d=json.loads(open('gpurun_out/b_w4r_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['runs'])"
done
for v in 0 1; do
TD3_W4=$v timeout -k 10 200 python3 bench.py --config pendulum --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/b_w4p_$v.json 2>/dev/null; echo "pendulum w4=$v rc=$?"; python3 -c "
import json;d=json.loads(open('gpurun_out/b_w4p_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['runs'])"
done
