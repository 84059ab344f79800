# split-K: pipelined walk at the 128-VGPR budget, and a lower matrix weight (TD3_DWSK_WM=2: 2 per matrix step)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for cfg in "2 6" "2 2" "0 2" "0 6"; do
  set -- $cfg
  TD3_DWSK_ORDER=$1 TD3_DWSK_WM=$2 timeout -k 10 200 python3 bench.py --config humanoid --steps 300 --warmup 30 --runs 3 --no-cpu-baseline > gpurun_out/hum_k_o$1_wm$2.json 2> gpurun_out/hum_k_o$1_wm$2.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hum_k_o$1_wm$2.json'));print('order $1 wm $2',d['value'],d['runs'],{k:v for k,v in d['stage_us'].items() if 'dw' in k})"
done
