#!/usr/bin/env python3
"""Fit the measured shard-time model of bench.py (`measured_cap`) to emulated multi-GPU
shard timings: T(shard) = T0 + kappa * cost, least squares over every emulated shard and
the whole model (bench.py --emulate-world N, JSON lines carrying shard_cost / total_cost),
one fit per model. Writes profiles/r04_shard_model.json with the fit and its largest
relative error on the points it was fitted to.

usage: tools/fit_shard_model.py EMULATION.json [...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pts = {}
src = {}
for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "shard_cost" not in d:
            continue
        m = d["model"]
        pts.setdefault(m, [])
        pts[m] += [(c, t) for c, t in zip(d["shard_cost"], d["shard_ms_per_sweep"]) if c > 0]
        pts[m].append((d["total_cost"], d["full_ms_per_sweep"]))
        src.setdefault(m, []).append(os.path.relpath(path, ROOT))
out = {}
for m, p in pts.items():
    c = np.array([x[0] for x in p])
    t = np.array([x[1] for x in p])
    A = np.stack([np.ones_like(c), c], 1)
    (t0, k), *_ = np.linalg.lstsq(A, t, rcond=None)
    err = np.abs((t0 + k * c) - t) / t
    out[m] = {"t0_ms": float(t0), "kappa_ms_per_cost": float(k), "max_rel_err": float(err.max()),
              "points": len(p), "sources": src[m]}
    print(m, out[m])
dst = os.path.join(ROOT, "profiles", "r04_shard_model.json")
old = {}
if os.path.exists(dst):
    old = json.load(open(dst))
old.update(out)
json.dump(old, open(dst, "w"), indent=1)
print("wrote", dst)
