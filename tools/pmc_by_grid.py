#!/usr/bin/env python3
"""Average counters per (kernel, grid size) from tools/pmc_groups.sh output.
usage: pmc_by_grid.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "k_"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("admmq::", "")
        if sub not in n:
            continue
        per[(n[:24], int(r["Grid_Size"]), r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (n, g, _), cs in per.items():
        for c, v in cs.items():
            agg[(n, g)][c].append(v)
for k in sorted(agg):
    print(k, {c: f"{sum(v)/len(v):.4g}" for c, v in sorted(agg[k].items())})
