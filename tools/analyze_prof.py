#!/usr/bin/env python3
"""Summarise a tools/profile.sh directory into profiles/<tag>_summary.md.

Per kernel: calls and average duration (kernel-trace stats), and per launch
HBM-side bytes from the PMC passes: FETCH_SIZE (KiB; doubled for gfx950, where it
reads half the bytes of a wide coalesced stream - MI355X_MICROARCH.md §HBM) and
WRITE_SIZE (KiB), plus SQ instruction counts.
"""
import csv
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("admmq::", "")[:60]


def read_counters(path):
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    if not os.path.exists(path):
        return agg, calls
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
            calls[k].add(row["Dispatch_Id"])
    return agg, calls


def main(d, tag, out):
    stats = os.path.join(d, "ktrace", "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    fetch, fcalls = read_counters(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write, wcalls = read_counters(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    sq, scalls = read_counters(os.path.join(d, "pmc_sq", "run_counter_collection.csv"))
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "Kernel-trace stats of `python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile` "
             "(C3 workload). PMC columns come from separate passes on a 20-iteration schedule "
             "(`--max-iter-admm 21`), per launch. FETCH bytes are FETCH_SIZE x 1024 x 2 (gfx950 correction), "
             "WRITE bytes WRITE_SIZE x 1024.", "",
             "| kernel | calls | avg us | share % | FETCH MB/launch (x2 corr.) | WRITE MB/launch | VALU instr/launch | MFMA instr/launch |",
             "|---|---|---|---|---|---|---|---|"]
    for r in rows[:25]:
        k = short(r["Name"])
        nf = max(len(fcalls.get(k, ())), 1)
        nw = max(len(wcalls.get(k, ())), 1)
        ns = max(len(scalls.get(k, ())), 1)
        fb = fetch[k].get("FETCH_SIZE", 0.0) * 1024 * 2 / nf / 1e6 if k in fetch else float("nan")
        wb = write[k].get("WRITE_SIZE", 0.0) * 1024 / nw / 1e6 if k in write else float("nan")
        va = sq[k].get("SQ_INSTS_VALU", float("nan")) / ns if k in sq else float("nan")
        mf = sq[k].get("SQ_INSTS_MFMA", float("nan")) / ns if k in sq else float("nan")
        lines.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} | "
                     f"{fb:.2f} | {wb:.2f} | {va:.3g} | {mf:.3g} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    d = sys.argv[1]
    tag = sys.argv[2]
    main(d, tag, sys.argv[3] if len(sys.argv) > 3 else f"profiles/{tag}_summary.md")
