#!/usr/bin/env python3
"""Per-launch HBM traffic of each ADMM launch class from a tools/profile.sh directory.

bytes/launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), averaged over the class's
launches in the PMC passes (20 iterations of each mode, so every mode weighs equally,
like bench.py's sampled HIP-event timing). FETCH_SIZE is doubled: on gfx950 it reads
half the bytes of a wide coalesced stream (MI355X_MICROARCH.md, HBM section); FETCH
and WRITE come from separate passes. Writes profiles/<tag>_traffic.json, which bench.py
reads into roofline.traffic.
usage: tools/traffic_json.py gpurun_out/prof_<tag> <tag>
"""
import csv
import json
import os
import sys
from collections import defaultdict

CLASSES = {"gemm": ("k_gemm",), "sse": ("k_mse_",), "finalize": ("k_finalize_admm",)}


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
    fetch, fn = per_dispatch(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, wn = per_dispatch(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {"source": f"gpurun_out/prof_{tag} (tools/profile.sh), summarised in profiles/{tag}_summary.md",
           "formula": "2*FETCH_SIZE + WRITE_SIZE per launch (gfx950 FETCH correction), separate PMC passes",
           "classes": {}}
    for cls, pref in CLASSES.items():
        fv = [v for k, v in fetch.items() if fn[k].startswith(pref)]
        wv = [v for k, v in write.items() if wn[k].startswith(pref)]
        if not fv or not wv:
            continue
        f_avg, w_avg = sum(fv) / len(fv), sum(wv) / len(wv)
        res["classes"][cls] = {"fetch_bytes": 2 * f_avg, "write_bytes": w_avg, "bytes_per_launch": 2 * f_avg + w_avg,
                               "launches": [len(fv), len(wv)]}
    os.makedirs("profiles", exist_ok=True)
    with open(os.path.join("profiles", f"{tag}_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
