set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drift.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p4.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/p4.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
TD3_L0R16_PAIR=$v timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/b_pair_$v.json 2>/dev/null; echo "bench pair=$v rc=$?"; python3 -c "
import json;d=json.loads(open('gpurun_out/b_pair_$v.json').read().strip().splitlines()[-1]);s=d['stage_us'];print(d['value'],d['runs']);print({k:v for k,v in s.items() if 'TF' in k or 'F_fwd01' in k})"
done
