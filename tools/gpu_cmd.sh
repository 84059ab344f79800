set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_w4.py tests/test_gpu_data_parallel.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pw4.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pw4.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/b_c2.json 2>/dev/null; echo "c2 rc=$? $(python3 -c "
import json;d=json.loads(open('gpurun_out/b_c2.json').read().strip().splitlines()[-1]);print(d['value'])")"
for r in 1 2; do for v in base ks0; do
  if [ $v = base ]; then lib=td3_amd/libtd3hip.so; else lib=tools/exp/libtd3hip_$v.so; fi
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/b_c2_${v}_$r.json 2>/dev/null; echo "c2 $v rc=$? $(python3 -c "
import json;d=json.loads(open('gpurun_out/b_c2_${v}_$r.json').read().strip().splitlines()[-1]);print(d['value'])")"
done; done
