#!/bin/bash
# Knockout A/B (GPU box): the C2 bench (2000 steps) and its rocprofv3 kernel stats with the default
# library and TD3_KO_* experiment builds (tools/build_exp.sh; wrong results, timing only).
#   tools/gpu_ko.sh koall [ko1 ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for v in base "$@" base "$@"; do
  if [ $v = base ]; then lib=td3_amd/libtd3hip.so; else lib=tools/exp/libtd3hip_$v.so; fi
  TD3_LIB=$lib timeout -k 10 200 python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-roofline > gpurun_out/kob_$v.json 2> gpurun_out/kob_$v.err
  rc=$?; [ $rc -ne 0 ] && { echo "$v bench rc=$rc"; tail -5 gpurun_out/kob_$v.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('gpurun_out/kob_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'])"
done
for v in base "$@"; do
  if [ $v = base ]; then lib=td3_amd/libtd3hip.so; else lib=tools/exp/libtd3hip_$v.so; fi
  TD3_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ko_$v -o run -- \
    python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-roofline > gpurun_out/ko_$v.json 2> gpurun_out/ko_$v.err
  rc=$?; echo "$v prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/ko_$v.err; exit $rc; }
done
python3 - "$@" <<'PY'
import csv, glob, sys
def load(v):
    f = glob.glob(f"gpurun_out/ko_{v}/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"].split("(")[0][:44]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f))}
vs = ["base"] + sys.argv[1:]
d = {v: load(v) for v in vs}
for k, (n, t) in sorted(d["base"].items(), key=lambda x: -x[1][0] * x[1][1]):
    if n < 100: continue
    print(f"{k:46s} {n:5d} " + " ".join(f"{d[v].get(k, (0, 0))[1]:7.2f}" for v in vs))
PY
