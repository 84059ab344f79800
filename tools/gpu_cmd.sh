set -o pipefail
F=gpurun_out/g13
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for i in 1 2 3; do
for st in 0 1; do
BENCH_SETTLE_MS=$st timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $F/bd_$st$i.json 2> $F/bd_$st$i.err || exit 1
python3 -c "import json;d=json.loads(open('$F/bd_$st$i.json').read().strip().splitlines()[-1]);print('settle $st', d['value'], d['runs'])"
done; done
