#!/usr/bin/env python3
"""Per-kernel table from scripts/pmc_kernels.sh output: median counter value
per (kernel, grid) over dispatches, plus derived per-wave figures."""
import collections
import csv
import glob
import os
import statistics
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "gpurun_out", "pmck")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, "*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            name = name.replace("void ", "")
            key = f"{name}@{r['Grid_Size']}"
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = ("k_decode", "k_encode")
for k in sorted(vals):
    if not any(w in k for w in want):
        continue
    v = {c: statistics.median(x) for c, x in vals[k].items()}
    waves = v.get("SQ_WAVES", 0) or 1
    line = [k[:70]]
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_VMEM_WR", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
              "SQ_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "FETCH_SIZE",
              "WRITE_SIZE"):
        if c in v:
            per = v[c] / waves if c.startswith("SQ_") and c not in ("SQ_WAVES", "SQ_BUSY_CYCLES") else v[c]
            line.append(f"{c.replace('SQ_', '')}={per:.4g}")
    print("  ".join(line))
