#!/usr/bin/env python3
"""Per-dispatch averages of the PMC passes written by tools/pmc_render.sh / pmc_sweep.sh:
    python tools/pmc_table.py gpurun_out/pmcr [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else ""
tab = defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
    variant = os.path.basename(os.path.dirname(f)).rsplit("_", 1)[0]
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"] or "mpiv" not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in per.items():
        tab[variant][c] = sum(d.values()) / len(d)
names = sorted({c for v in tab.values() for c in v})
vs = sorted(tab)
print(f"{'counter':28s}" + "".join(f"{v:>16s}" for v in vs))
for c in names:
    print(f"{c:28s}" + "".join(f"{tab[v].get(c, float('nan')):16.4g}" for v in vs))
