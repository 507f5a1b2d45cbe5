#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace CSV (diagnostics).

For each ordered pair of kernel classes (previous -> next, names shortened to the text
before '<' / '('), prints the count and the mean / median gap between the previous
kernel's end and the next one's start, and each class's mean duration.
usage: tools/ktrace_gaps.py gpurun_out/prof_<tag>_<model>/ktrace"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("admmq::", "")
    return n.split("(")[0].split("<")[0].strip()


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    gaps = defaultdict(list)
    dur = defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = (s1 - e0) / 1e3
        if 0 <= g < 100:   # same stream, back to back (longer gaps: host work)
            gaps[(n0, n1)].append(g)
    for s, e, n in rows:
        dur[n].append((e - s) / 1e3)
    print(f"{len(rows)} dispatches from {len(files)} file(s)")
    print("gap (us) previous -> next: count, mean, median")
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:12]:
        print(f"  {a:>22s} -> {b:<22s} {len(v):7d} {statistics.mean(v):7.2f} {statistics.median(v):7.2f}")
    print("duration (us): count, mean")
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:8]:
        print(f"  {n:<24s} {len(v):7d} {statistics.mean(v):9.2f}")


if __name__ == "__main__":
    main()
