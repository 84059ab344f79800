set -o pipefail
F=gpurun_out/final2
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 python3 bench.py > $F/bench.json 2> $F/bench.err; echo "bench rc=$?"
for i in 1 2 3; do timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_driver_$i.json 2> $F/bench_driver_$i.err; echo "driver $i rc=$?"; done
