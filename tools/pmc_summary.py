#!/usr/bin/env python3
"""Per-kernel averages of every counter collected by tools/pmc.sh (one row per kernel)."""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("admmq::", "").replace("void ", "")[:28]
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        for c, v in cs.items():
            vals[k][c].append(v)
keys = [k for k in vals if k.startswith(("k_gemm", "k_mse", "k_finalize"))]
for k in sorted(keys):
    print(f"== {k}")
    for c in sorted(vals[k]):
        xs = vals[k][c]
        print(f"   {c:28s} {sum(xs)/len(xs):14.1f}")
