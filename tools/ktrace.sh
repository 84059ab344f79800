#!/bin/bash
# Kernel-trace summary of a bench run (GPU box).  Usage: tools/ktrace.sh TAG "bench args" [lib.so]
set -o pipefail
tag=$1; args=$2; lib=${3:-}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ -n "$lib" ]; then export TD3_LIB=$lib; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o run -- python3 bench.py $args > gpurun_out/kt_$tag.log 2>&1 || { echo "ktrace $tag failed"; tail -5 gpurun_out/kt_$tag.log; exit 1; }
python3 - "$tag" <<'PY'
import csv, collections, sys, glob
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/kt_{tag}/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = (r["Kernel_Name"].replace("void ", "")[:48], r["Grid_Size_X"], r["Grid_Size_Y"])
    d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print(f"{tag} {k[0]:48s} grid {k[1]:>7s}x{k[2]:<2s} n={len(v):4d} avg {sum(v)/len(v):9.1f} us")
PY
