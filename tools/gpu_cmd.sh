set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for i in 1 2 3 4; do for g in 1 0; do
  BENCH_GC=$g timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/b_gc${g}_$i.json 2>/dev/null; echo "gc=$g rc=$? $(python3 -c "
import json;d=json.loads(open('gpurun_out/b_gc${g}_$i.json').read().strip().splitlines()[-1]);print(d['value'], [round(x) for x in d['runs']])")"
done; done
