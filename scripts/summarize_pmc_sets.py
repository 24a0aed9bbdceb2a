#!/usr/bin/env python3
"""Per-kernel medians of every counter in a directory of rocprofv3 --pmc
passes (p1/, p2/, ... as written by scripts/pmc_passes.sh), one line per
kernel and counter.  Usage: summarize_pmc_sets.py DIR [kernel-substring]"""
import collections
import csv
import glob
import os
import statistics
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"),
                             recursive=True)):
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            name = name.replace("void ", "")
            if filt not in name:
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    print(k)
    for c, v in sorted(vals[k].items()):
        print(f"   {c:24s} {statistics.median(v):16.0f}  (n={len(v)})")
