#!/usr/bin/env python3
"""SURVEY §8(f)3 timing: quant + low-rank ADMM at the reference notebook's measured
configuration (notebooks/LlamaADMMQuant.ipynb cell 15: layer 0 q_proj 4096 x 4096,
4-bit tensor_minmax, rank 8, 100 outer iterations of admm_iteration(max_iter=50) for
the quantized part and for the low-rank part; 2 h 32 min 18 s wall on an A100,
:510-511), on a synthetic Llama-7B weight of that shape (N(0, 0.02^2), admmq.synthetic).

Runs, on one MI355X:
  * the full 100-outer-iteration loop with the device rank projection
    (admmq.lowrank.SubspaceProjector: warm-started block subspace iteration on the
    device, thin GEMMs + a 16 x 4096 SVD per sweep), wall-timed;
  * the reference's exact projection (torch.linalg.svd of the 4096 x 4096 iterate, the
    notebook's project_rank) timed on a bounded sample: SVD calls, then extrapolated
    to the exact-projection loop's projection count;
  * agreement of the two projections on the loop's final low-rank target W - W_q.
Prints one JSON line.  usage: tools/lowrank_bench.py [--outer 100] [--svd-sample 4]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "admm-quantization_amd")]
import torch  # noqa: E402
from functools import partial  # noqa: E402

from admmq import synthetic  # noqa: E402
from admmq.lowrank import SubspaceProjector, admm_iteration, project_rank  # noqa: E402
from admmq.quantization import quantize_tensor  # noqa: E402

A100_SECONDS = 2 * 3600 + 32 * 60 + 18


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--outer", type=int, default=100)
    ap.add_argument("--inner", type=int, default=50)
    ap.add_argument("--rank", type=int, default=8)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--svd-sample", type=int, default=4, help="exact SVD projections timed (extrapolated)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    spec = synthetic.llama_layers()[0]
    W = torch.from_numpy(synthetic.layer_weight(spec, 0)).to(dev)
    g = torch.Generator().manual_seed(42)
    quant = partial(quantize_tensor, qscheme="tensor_minmax", bits=a.bits)
    nw = torch.linalg.norm(W)

    X0 = torch.randn(*W.shape, generator=g).to(dev)
    # exact SVD projection: timed sample
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.svd_sample):
        project_rank(X0 + 1e-3 * torch.randn_like(X0), a.rank)
    torch.cuda.synchronize()
    svd_s = (time.perf_counter() - t0) / a.svd_sample

    # the notebook loop with the device projection
    W_q = torch.randn(*W.shape, generator=g).to(dev)
    U_q = torch.zeros_like(W_q)
    proj = SubspaceProjector(a.rank, seed=42)
    W_r = proj(torch.randn(*W.shape, generator=g).to(dev))
    U_r = torch.zeros_like(W_r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist, nq, nr = [], 0, 0
    for i in range(a.outer):
        W_q, U_q, iq = admm_iteration(W_q, U_q, W, W_r, quant, rho=1.0, max_iter=a.inner, return_iters=True)
        W_r, U_r, ir = admm_iteration(W_r, U_r, W, W_q, proj, rho=1.0, max_iter=a.inner, return_iters=True)
        nq += iq
        nr += ir
        if i % 10 == 0 or i == a.outer - 1:
            hist.append(round(float(torch.linalg.norm(W - W_r - W_q) / nw), 4))
            print(f"outer {i}: rel {hist[-1]}", flush=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # agreement of the device projection with the exact truncation on the loop's own
    # low-rank target W - W_q (fresh projector, cold start) and that matrix's spectral gap
    Xe = (W - W_q).contiguous()
    exact = project_rank(Xe, a.rank)
    approx = SubspaceProjector(a.rank, seed=1)(Xe)
    agree = float(torch.linalg.norm(approx - exact) / torch.linalg.norm(exact))
    sv = torch.linalg.svdvals(Xe)
    gap = float(sv[a.rank - 1] / sv[a.rank])
    out = {"config": "LlamaADMMQuant.ipynb cell 15: q_proj 4096x4096 synthetic N(0,0.02^2), 4-bit tensor_minmax, "
                     f"rank {a.rank}, {a.outer} outer x admm_iteration(max_iter={a.inner}) x 2",
           "device_projection": "SubspaceProjector (warm-started block subspace iteration, k = rank + 8)",
           "wall_s": wall, "a100_reference_wall_s": A100_SECONDS, "speedup_vs_a100_notebook": A100_SECONDS / wall,
           "inner_iterations": {"quant": nq, "rank": nr}, "subspace_sweeps_mean": sum(proj.sweeps) / len(proj.sweeps),
           "rel_history": hist, "exact_svd_projection_s": svd_s,
           "exact_svd_loop_estimate_s": svd_s * nr, "device_vs_exact_projection_rel": agree,
           "sigma_r_over_sigma_r1": gap}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
