set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TD3_LIB=tools/exp/libtd3hip_tl.so timeout -k 10 200 python3 tools/tl_probe.py > gpurun_out/tl_r16.txt 2>&1; echo "tl rc=$?"; grep -v amdgpu.ids gpurun_out/tl_r16.txt | head -10
for v in 1 0; do
TD3_L0R16=$v timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/b_r16_$v.json 2>/dev/null; echo "bench r16=$v rc=$?"; python3 -c "
import json;d=json.loads(open('gpurun_out/b_r16_$v.json').read().strip().splitlines()[-1]);print(d['value'],d['runs'])"
done
