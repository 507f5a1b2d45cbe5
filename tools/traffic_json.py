#!/usr/bin/env python3
"""Per-launch HBM traffic of each ADMM launch class from a tools/profile.sh directory.

bytes/launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), averaged over the class's
launches in the PMC passes (20 iterations of each mode, so every mode weighs equally,
like bench.py's sampled HIP-event timing). FETCH_SIZE is doubled: on gfx950 it reads
half the bytes of a wide coalesced stream (MI355X_MICROARCH.md, HBM section); FETCH
and WRITE come from separate passes. Writes profiles/<tag>_traffic.json, which bench.py
reads into roofline.traffic.
usage: tools/traffic_json.py gpurun_out/prof_<tag> <tag> [model] [split|fp32]
(writes profiles/<tag>_<model>_traffic.json)
"""
import csv
import json
import os
import sys
from collections import defaultdict

# bench.py's launch classes (ADMMQ_PROF_*) by kernel-name prefix
CLASSES = {"gemm": ("k_gemm<", "k_gemm_f32b<"), "gemm_thin": ("k_thin_solve",), "search": ("k_mse_hist", "k_mse_sse", "k_mse_select"),
           "small": ("k_mse_small_admm",), "finalize": ("k_finalize_admm",), "thin_loop": ("k_thin_loop",)}


def per_dispatch(path, counter):
    out = defaultdict(float)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("admmq::", "")
            out[r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024.0
            names[r["Dispatch_Id"]] = n
    return out, names


def main():
    d, tag = sys.argv[1], sys.argv[2]
    model = sys.argv[3] if len(sys.argv) > 3 else "resnet18"
    solve = sys.argv[4] if len(sys.argv) > 4 else "split"
    fetch, fn = per_dispatch(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, wn = per_dispatch(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {"source": f"{os.path.normpath(d)} (tools/profile.sh), summarised in profiles/{tag}_{model}_summary.md",
           "formula": "2*FETCH_SIZE + WRITE_SIZE per launch (gfx950 FETCH correction), separate PMC passes",
           "model": model, "split": solve == "split", "classes": {}}
    for cls, pref in CLASSES.items():
        fv = [v for k, v in fetch.items() if fn[k].startswith(pref)]
        wv = [v for k, v in write.items() if wn[k].startswith(pref)]
        if not fv or not wv:
            continue
        f_avg, w_avg = sum(fv) / len(fv), sum(wv) / len(wv)
        res["classes"][cls] = {"fetch_bytes": 2 * f_avg, "write_bytes": w_avg, "bytes_per_launch": 2 * f_avg + w_avg,
                               "launches": [len(fv), len(wv)]}
    os.makedirs("profiles", exist_ok=True)
    with open(os.path.join("profiles", f"{tag}_{model}_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
