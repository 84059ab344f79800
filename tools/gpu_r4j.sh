# split-K partition weights (TD3_DWSK_WM: matrix-step weight 2 + WM/4 against 1 per vector step) x walk
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for o in 0 2; do for wm in 6 8 10 12; do
  TD3_DWSK_ORDER=$o TD3_DWSK_WM=$wm timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_o${o}_wm$wm.json 2> gpurun_out/hum_o${o}_wm$wm.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_o${o}_wm$wm.json'));print('order $o wm $wm',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done; done
