#!/usr/bin/env python3
"""Wall time per ADMM iteration of one mode's batched problems (bench shapes),
two-stage vs exhaustive MSE search (diagnostics for the per-mode search choice)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "admm-quantization_amd"))
import torch  # noqa: E402
from admmq import _lib, synthetic  # noqa: E402
from admmq.admm import admm_iteration_batched  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=201)
ap.add_argument("--model", default="resnet18")
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _lib.load()
for mode in range(3):
    g = torch.Generator().manual_seed(0)
    probs = []
    for s in synthetic.MODELS[a.model]():
        if mode >= len(s.shape):
            continue
        R = s.rank()
        I = s.shape[mode]
        B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
        G = (B @ B.T + 0.5 * torch.eye(R)).to(dev)
        F = torch.randn(I, R, generator=g).to(dev)
        H = torch.randn(I, R, generator=g).to(dev) * 0.1
        probs.append((H, torch.zeros(I, R, device=dev), F, G))
    for ex in (0, 1):
        lib.admmq_set_exhaustive_search(ex)
        admm_iteration_batched([(h, u.clone(), f, gg) for h, u, f, gg in probs], 3, 0.0, 4,
                               "tensor_mseminmax_symmetric", check_spd=False)
        torch.cuda.synchronize()
        ts = []
        for its in (2, a.iters):
            t0 = time.perf_counter()
            admm_iteration_batched([(h, u.clone(), f, gg) for h, u, f, gg in probs], its, 0.0, 4,
                                   "tensor_mseminmax_symmetric", check_spd=False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        per = (ts[1] - ts[0]) / (a.iters - 2) * 1e6
        print(f"mode {mode} exhaustive={ex}: {per:7.1f} us per iteration ({len(probs)} problems)")
    lib.admmq_set_exhaustive_search(0)
