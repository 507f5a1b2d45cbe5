#!/usr/bin/env python3
"""F10: the reference's quant + low-rank ADMM loop at a mid size over many outer
iterations (survey container only; python3 -B tests/golden/gen_f10_lowrank.py).

scripts/factorize_lowrank.py (imported with bitsandbytes stubbed, gen_golden.import_lowrank)
runs its alternating loop (:156-170: admm_iteration(W_q, ...quantize...) then
admm_iteration(W_r, ...project_rank...), inner max_iter 50, rho 1) on a 1024 x 1024
synthetic weight W ~ N(0, 0.02^2) with 4-bit tensor_minmax and rank 8, for 30 outer
iterations, from its 'random' init (W_q = randn, W_r = project_rank(randn)). The inputs are
regenerated from a torch CPU generator seed; W_r0 is the reference's own project_rank of
the seeded draw (torch CPU SVD). Stored: the per-outer-iteration rel = ||W - W_q - W_r|| /
||W|| (the reference's rel_admm_diff, :161-162), and the same loop re-run from starts ~1 ulp
away (W_r0 from a float64 SVD; one ulp on a random 1 % of W_r0's elements, two seeds) and at
1 CPU thread: the per-iteration [min, max] over the five runs is the reference's own band.
Data only (JSON): tests/golden/f10_lowrank.json."""
import json
import os
import sys
import time
from functools import partial

sys.dont_write_bytecode = True
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden  # noqa: E402

SEED, N, SCALE, BITS, RANK, QS, OUTER = 1010, 1024, 0.02, 4, 8, "tensor_minmax", 30


def inputs():
    g = torch.Generator().manual_seed(SEED)
    W = torch.randn(N, N, generator=g) * SCALE
    Wq0 = torch.randn(N, N, generator=g)
    Wr0_raw = torch.randn(N, N, generator=g)
    return W, Wq0, Wr0_raw


def run(lowrank, ref_quant, W, Wq, Wr):
    qf = partial(ref_quant.quantize_tensor, qscheme=QS, bits=BITS)
    pf = partial(lowrank.project_rank, rank=RANK)
    Uq, Ur = torch.zeros_like(Wq), torch.zeros_like(Wr)
    rel = []
    for i in range(OUTER):
        t0 = time.time()
        Wq, Uq = lowrank.admm_iteration(Wq, Uq, W, Wr, qf, rho=1.0)
        Wr, Ur = lowrank.admm_iteration(Wr, Ur, W, Wq, pf, rho=1.0)
        rel.append(float(torch.linalg.norm(W - Wr - Wq) / torch.linalg.norm(W)))
        print(f"outer {i}: rel {rel[-1]:.6f} ({time.time() - t0:.1f}s)", flush=True)
    return rel


def main():
    torch.set_num_threads(8)
    _, ref_quant = gen_golden.import_reference("/root/reference")
    lowrank = gen_golden.import_lowrank("/root/reference")
    W, Wq0, Wr0_raw = inputs()
    Wr0 = lowrank.project_rank(Wr0_raw, RANK)
    rel = run(lowrank, ref_quant, W, Wq0.clone(), Wr0.clone())
    # the same loop from starts ~1 ulp away: W_r0 from a float64 SVD, and W_r0 with one ulp
    # added to a random 1 % of its elements (two seeds); and the reference at 1 CPU thread
    U, S, Vt = torch.linalg.svd(Wr0_raw.double())
    starts = {"fp64_svd_start": (U[:, :RANK] @ torch.diag(S[:RANK]) @ Vt[:RANK]).float()}
    for sd in (1, 2):
        g = torch.Generator().manual_seed(sd)
        sel = torch.rand(N, N, generator=g) < 0.01
        starts[f"ulp_start_seed{sd}"] = torch.where(sel, torch.nextafter(Wr0, torch.full_like(Wr0, float("inf"))), Wr0)
    pert = {}
    for k, w0 in starts.items():
        pert[k] = {"start_rel": float(torch.linalg.norm(w0 - Wr0) / torch.linalg.norm(Wr0)),
                   "rel_history": run(lowrank, ref_quant, W, Wq0.clone(), w0)}
    torch.set_num_threads(1)
    pert["threads1"] = {"start_rel": 0.0, "rel_history": run(lowrank, ref_quant, W, Wq0.clone(), Wr0.clone())}
    torch.set_num_threads(8)
    allh = [rel] + [v["rel_history"] for v in pert.values()]
    out = {"generator": "tests/golden/gen_f10_lowrank.py", "reference": "scripts/factorize_lowrank.py:80-101,156-170",
           "torch": torch.__version__, "threads": 8, "seed": SEED, "shape": [N, N], "scale": SCALE, "bits": BITS,
           "rank": RANK, "qscheme": QS, "outer": OUTER, "inner_max_iter": 50, "rho": 1.0,
           "inputs": "torch.Generator().manual_seed(seed): W = randn(N, N) * scale, W_q0 = randn(N, N), "
                     "W_r0 = project_rank(randn(N, N), rank) (reference, torch CPU SVD)",
           "rel_history": rel, "perturbed": pert,
           "band_min": [min(h[i] for h in allh) for i in range(OUTER)],
           "band_max": [max(h[i] for h in allh) for i in range(OUTER)],
           "max_abs_diff_perturbed": max(abs(a - b) for h in allh[1:] for a, b in zip(rel, h))}
    with open(os.path.join(HERE, "f10_lowrank.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("F10:", out["max_abs_diff_perturbed"], rel[0], rel[-1], [round(b - a, 4) for a, b in zip(out["band_min"], out["band_max"])])


if __name__ == "__main__":
    main()
