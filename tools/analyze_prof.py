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
    tcc, tcalls = read_counters(os.path.join(d, "pmc_tcc", "run_counter_collection.csv"))
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "Kernel-trace stats of `python3 bench.py --model <model> --steps 2 --warmup 1 --no-cpu-baseline --no-profile` "
             f"(directory `{d}`). PMC columns come from separate passes on a 20-iteration schedule "
             "(`--max-iter-admm 21`), per launch. FETCH bytes are FETCH_SIZE x 1024 x 2 (gfx950 correction), "
             "WRITE bytes WRITE_SIZE x 1024.", "",
             "MFMA busy % (GRBM) = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) (GRBM_GUI_ACTIVE sums "
             "the 8 XCDs; MI355X_MICROARCH.md). It reads LOW on short dispatches: GRBM_GUI_ACTIVE / 8 over the "
             "kernel-trace wall time (column GRBM GHz) comes out above any clock the chip runs (MI355X_MICROARCH.md, "
             "DVFS: the quotient reads high below ~0.3 ms), i.e. the denominator counts cycles outside the kernel. "
             "cyc/MFMA = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA (64 for v_mfma_f32_32x32x2_f32: 4096 flops at "
             "64 flops/cycle/SIMD). MFMA busy % (wall) = SQ_VALU_MFMA_BUSY_CYCLES / (wall x 2.4 GHz x 1024 SIMDs): "
             "with 64 cycles per MFMA this is the MFMA flop rate over the 157.3 TF/s peak (padding included). "
             "LDS conflicts are SQ_LDS_BANK_CONFLICT extra cycles per LDS instruction. "
             "L2 hit % = TCC_HIT / (TCC_HIT + TCC_MISS).", "",
             "| kernel | calls | avg us | share % | FETCH MB/launch (x2 corr.) | WRITE MB/launch | VALU instr/launch | "
             "MFMA instr/launch | cyc/MFMA | GRBM GHz | MFMA busy % (GRBM) | MFMA busy % (wall) | LDS confl./instr | L2 hit % |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows[:25]:
        k = short(r["Name"])
        nf = max(len(fcalls.get(k, ())), 1)
        nw = max(len(wcalls.get(k, ())), 1)
        ns = max(len(scalls.get(k, ())), 1)
        fb = fetch[k].get("FETCH_SIZE", 0.0) * 1024 * 2 / nf / 1e6 if k in fetch else float("nan")
        wb = write[k].get("WRITE_SIZE", 0.0) * 1024 / nw / 1e6 if k in write else float("nan")
        va = sq[k].get("SQ_INSTS_VALU", float("nan")) / ns if k in sq else float("nan")
        mf = sq[k].get("SQ_INSTS_MFMA", float("nan")) / ns if k in sq else float("nan")
        nan = float("nan")
        busy = busy_w = cyc = ghz = nan
        wall_s = float(r["AverageNs"]) * 1e-9
        if k in sq and sq[k].get("GRBM_GUI_ACTIVE"):
            busy = 100.0 * sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES", nan) / (sq[k]["GRBM_GUI_ACTIVE"] / 8 * 1024)
            ghz = sq[k]["GRBM_GUI_ACTIVE"] / ns / 8 / wall_s / 1e9
        if k in sq and sq[k].get("SQ_INSTS_MFMA"):
            cyc = sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES", nan) / sq[k]["SQ_INSTS_MFMA"]
            busy_w = 100.0 * sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES", nan) / ns / (wall_s * 2.4e9 * 1024)
        confl = sq[k].get("SQ_LDS_BANK_CONFLICT", nan) / sq[k]["SQ_INSTS_LDS"] if k in sq and sq[k].get("SQ_INSTS_LDS") else nan
        hit = nan
        if k in tcc:
            h, m = tcc[k].get("TCC_HIT_sum", 0.0), tcc[k].get("TCC_MISS_sum", 0.0)
            hit = 100.0 * h / (h + m) if h + m else nan
        lines.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} | "
                     f"{fb:.2f} | {wb:.2f} | {va:.3g} | {mf:.3g} | {cyc:.1f} | {ghz:.2f} | {busy:.1f} | {busy_w:.1f} | "
                     f"{confl:.2f} | {hit:.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    d = sys.argv[1]
    tag = sys.argv[2]
    main(d, tag, sys.argv[3] if len(sys.argv) > 3 else f"profiles/{tag}_summary.md")
