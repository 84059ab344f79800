set -o pipefail
B="python3 bench.py --steps 3000 --warmup 200 --no-cpu-baseline --no-roofline"
run() { echo "$1: $(timeout -k 10 120 env $2 $B $3 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')"; }
run base "X=1"
run eager "X=1" --eager
run devkernarg "HIP_FORCE_DEV_KERNARG=1"
run pktcap0 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"
run pktcap1 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"
run base2 "X=1"
