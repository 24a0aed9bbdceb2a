#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by
(kernel, grid size): calls, mean / median / min microseconds, VGPRs.
Usage: kernel_table.py run_kernel_trace.csv [name-substring]"""
import collections
import csv
import statistics
import sys

rows = collections.defaultdict(list)
meta = {}
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0]
    if filt not in name:
        continue
    key = (name, int(r["Grid_Size_X"]))
    rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    meta[key] = (r["VGPR_Count"], r["LDS_Block_Size"])
print(f"{'kernel':44s} {'grid':>10s} {'calls':>6s} {'mean':>9s} {'median':>9s} {'min':>9s} vgpr lds")
for key in sorted(rows, key=lambda k: -sum(rows[k])):
    d = rows[key]
    print(f"{key[0][:44]:44s} {key[1]:10d} {len(d):6d} {statistics.mean(d):9.1f} "
          f"{statistics.median(d):9.1f} {min(d):9.1f} {meta[key][0]:>4s} {meta[key][1]}")
