#!/usr/bin/env python3
"""Per-kernel PMC summary of a scripts/pmc_passes.sh directory as JSON: the
median of every counter per (kernel, grid), with the gfx950 corrections of
MI355X_MICROARCH.md (FETCH_SIZE doubled, both in KiB) and per-wave figures.
Usage: pmc_table.py DIR OUT.json [kernel-substring ...]"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

src, dst = sys.argv[1], sys.argv[2]
want = sys.argv[3:] or ["k_"]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"),
                             recursive=True)):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        if not any(w in name for w in want):
            continue
        vals[f"{name}@grid{r['Grid_Size']}"][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in sorted(vals.items()):
    med = {c: statistics.median(v) for c, v in cs.items()}
    waves = med.get("SQ_WAVES") or 1
    e = {"counters_median": med}
    if "FETCH_SIZE" in med:
        e["hbm_read_bytes"] = 2 * med["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in med:
        e["hbm_write_bytes"] = med["WRITE_SIZE"] * 1024
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_VMEM_WR"):
        if c in med:
            e[c.replace("SQ_INSTS_", "") + "_per_wave"] = med[c] / waves
    out[k] = e
json.dump({"source": src, "corrections": "hbm_read = 2 x FETCH_SIZE KiB, hbm_write = WRITE_SIZE KiB",
           "kernels": out}, open(dst, "w"), indent=1)
for k, e in out.items():
    print(k, {x: round(y, 1) for x, y in e.items() if not isinstance(y, dict)})
