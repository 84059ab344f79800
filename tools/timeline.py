#!/usr/bin/env python3
"""Per-kernel timeline of a rocprofv3 kernel trace: durations and the idle gap before each
kernel, averaged over the steady-state steps.  Usage: tools/timeline.py trace.csv [first_kernel_substr]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "gather_kernel"
ks = [(r["Kernel_Name"].replace("void ", "").split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
      for r in rows]
# split into steps at each marker kernel
steps, cur = [], []
for k in ks:
    if mark in k[0] and cur:
        steps.append(cur)
        cur = []
    cur.append(k)
steps = steps[len(steps) // 2:]           # steady state: second half
sig = collections.defaultdict(list)
for s in steps:
    sig[tuple(k[0] for k in s)].append(s)
for names, group in sorted(sig.items(), key=lambda kv: -len(kv[1]))[:2]:
    n = len(group)
    print(f"== {n} steps of {len(names)} kernels")
    tot_d = tot_g = 0.0
    for i, nm in enumerate(names):
        d = sum((s[i][2] - s[i][1]) for s in group) / n / 1e3
        if i == 0:
            g = 0.0
        else:
            g = sum((s[i][1] - s[i - 1][2]) for s in group) / n / 1e3
        tot_d += d
        tot_g += g
        print(f"  {nm[:44]:44s} dur {d:7.2f}  gap {g:6.2f}")
    span = sum((s[-1][2] - s[0][1]) for s in group) / n / 1e3
    print(f"  sum dur {tot_d:.1f}  sum gaps {tot_g:.1f}  span {span:.1f} us")
# gap between steps
gaps = [steps[i + 1][0][1] - steps[i][-1][2] for i in range(len(steps) - 1)]
print(f"inter-step gap avg {sum(gaps) / len(gaps) / 1e3:.2f} us; step period "
      f"{(steps[-1][0][1] - steps[0][0][1]) / (len(steps) - 1) / 1e3:.2f} us")
