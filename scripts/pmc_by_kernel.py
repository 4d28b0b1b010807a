#!/usr/bin/env python3
"""Median per-dispatch PMC values per kernel from the pass directories of a rocprofv3 run
(scripts/prof_pipeline_pmc.sh), beside the kernel-trace averages; writes <dir>/pmc_by_kernel.md."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("usv::(anonymous namespace)::", "").split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {}
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        avg[r["Name"].replace("usv::(anonymous namespace)::", "").split("(")[0]] = float(r["AverageNs"]) / 1e3
lines = [f"# PMC medians per dispatch by kernel ({d})", ""]
for k in sorted(vals):
    if "usv" not in k and not any(x in k for x in ("remap", "hist", "equalize", "mask", "pack_map", "tile_box")):
        continue
    lines.append(f"## {k} ({avg.get(k, float('nan')):.2f} us avg)")
    for c in sorted(vals[k]):
        lines.append(f"  {c:40s} {statistics.median(vals[k][c]):14.6g}")
    lines.append("")
txt = "\n".join(lines)
open(os.path.join(d, "pmc_by_kernel.md"), "w").write(txt)
print(txt)
