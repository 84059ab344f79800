#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

Correction per /opt/skills/guides/MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE (KiB) reports
half the bytes of a wide coalesced read -> x2; WRITE_SIZE (KiB) is exact for 16-B stores.
Both counters count fabric-side traffic (Infinity-Cache hits included).

    python tools/pmc_summary.py gpurun_out/pmcf/run_counter_collection.csv \
        gpurun_out/pmcw/run_counter_collection.csv profiles/pmc_traffic.json
"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").strip()
        vals[name].append(float(r["Counter_Value"]))
    return vals


def main():
    fpath, wpath, out = sys.argv[1:4]
    f = per_kernel(fpath, "FETCH_SIZE")
    w = per_kernel(wpath, "WRITE_SIZE")
    res = {"source": {"fetch": fpath, "write": wpath},
           "correction": "fetch_bytes = 2 * FETCH_SIZE KiB * 1024 (gfx950 half-count); "
                         "write_bytes = WRITE_SIZE KiB * 1024",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb = 2 * 1024 * sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wb = 1024 * sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        res["kernels"][k] = {"launches_profiled": max(len(f.get(k, [])), len(w.get(k, []))),
                             "fetch_bytes_per_launch": round(fb),
                             "write_bytes_per_launch": round(wb),
                             "hbm_bytes_per_launch": round(fb + wb)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:45s} {v['launches_profiled']:5d}  fetch {v['fetch_bytes_per_launch']/1e6:8.3f} MB  "
              f"write {v['write_bytes_per_launch']/1e6:8.3f} MB")


if __name__ == "__main__":
    main()
