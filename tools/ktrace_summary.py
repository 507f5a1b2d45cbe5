#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace directory."""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("admmq::", "")
    if n.startswith("k_"):
        d[(n[:26], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    if len(v) >= 50:
        print(f"{k[0]:26s} grid {k[1]:8d} n {len(v):5d} avg {sum(v)/len(v):7.1f} min {min(v):7.1f} max {max(v):7.1f} us")
