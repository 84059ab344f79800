#!/bin/bash
# PMC passes over a bench command (GPU box).  Usage: tools/pmc_probe.sh TAG "bench args" "CTR1 CTR2 ..." ["CTR ..."]...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
tag=$1; args=$2; shift 2
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_${tag}_$i -o run -- python3 bench.py $args > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
python3 - "$tag" "$i" <<'PY'
import csv, collections, re, sys, glob
tag, n = sys.argv[1], int(sys.argv[2])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for k in range(1, n + 1):
    for f in glob.glob(f"gpurun_out/pmc_{tag}_{k}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").strip()
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, d in sorted(acc.items()):
    if not any(x in name for x in ("enc_", "gemm", "dw", "row_")):
        continue
    print(name, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
