# C2 launch policy in the driver's regime: direct launches (auto) vs hipGraph replay, long and short runs
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for L in auto graph; do
  timeout -k 10 200 python3 bench.py --launch $L --steps 2000 --warmup 100 --runs 3 --no-cpu-baseline --no-roofline > gpurun_out/c2_long_$L.json 2> gpurun_out/c2_long_$L.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c2_long_$L.json'));print('long $L',d['value'],d['runs'])"
  for i in 1 2 3; do
    timeout -k 10 200 python3 bench.py --launch $L --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/c2_short_${L}_$i.json 2> gpurun_out/c2_short_${L}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c2_short_${L}_$i.json'));print('short $L',d['value'],d['runs'])"
  done
done
