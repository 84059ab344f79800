set -o pipefail
B="python3 bench.py --steps 3000 --warmup 200 --no-cpu-baseline --no-roofline"
for m in auto graph eager auto; do
echo "$m: $(timeout -k 10 120 $B --launch $m | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')"
done
