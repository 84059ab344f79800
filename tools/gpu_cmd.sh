set -o pipefail
F=gpurun_out/final
mkdir -p $F
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TD3_LIB=tools/exp/libtd3hip_tl.so timeout -k 10 200 python3 tools/tl_probe.py > $F/timeline_halfcheetah.txt 2>&1; echo "tl hc rc=$?"
TL_SHAPE=376,17,1024 TD3_LIB=tools/exp/libtd3hip_tl.so timeout -k 10 200 python3 tools/tl_probe.py > $F/timeline_humanoid.txt 2>&1; echo "tl hum rc=$?"
for c in halfcheetah pendulum humanoid; do
  a=""; [ $c = humanoid ] && a="--steps 600 --warmup 50"
  timeout -k 10 500 python3 bench.py --config $c $a > $F/bench2_$c.json 2> $F/bench2_$c.err; echo "bench $c rc=$? $(tail -c 300 $F/bench2_$c.json | cut -c1-200)"
done
