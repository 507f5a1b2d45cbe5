"""ORACLE — test infrastructure only. torch-CPU port of the reference ADMM step, used
as ``bench.py``'s ``cpu_baseline`` (kind "port").

It keeps the reference's CPU cost structure so the baseline is representative of
``scripts/factorize.py`` run on host cores: per inner iteration one
``cholesky_solve`` (``source/admm.py:56``) and the 200-candidate search as 200
full-tensor passes with a float32 mean (``source/quantization.py:129-144``),
multi-threaded by torch. Pinned against the reference's own outputs in
``tests/test_host.py::test_torch_port_vs_reference_fixtures``. Nothing in the
product path imports this file.
"""
from __future__ import annotations

import torch


def quantize_mse(x: torch.Tensor, bits: int, num_attempts: int = 200) -> torch.Tensor:
    qmax = 2 ** (bits - 1)
    den = 2 * qmax - 1
    mx = torch.maximum(x.min().abs(), x.max().abs())
    cands = torch.linspace(0.2 * mx.item(), 1.2 * mx.item(), num_attempts)
    scales = (2 * cands) / den
    mses = torch.empty(num_attempts)
    for i in range(num_attempts):
        s = scales[i:i + 1]
        err = x - torch.clamp(torch.round(x / s), -qmax, qmax - 1) * s
        mses[i] = (err * err).mean()
    s = scales[int(torch.argmin(mses))].reshape(1)
    return torch.clamp(torch.round(x / s), -qmax, qmax - 1) * s


def admm_iteration(H, U, F, G, max_iter, eps, bits, num_attempts=200):
    """source/admm.py:51-67 on torch-CPU float32 (mse-minmax scheme)."""
    R = H.shape[1]
    rho = torch.trace(G) / R
    L = torch.linalg.cholesky(G + rho * torch.eye(R))
    U = U.clone()
    for _ in range(1, max_iter):
        HT = torch.cholesky_solve((F + rho * (H + U)).T, L).T
        Hp = H
        H = quantize_mse(HT - U, bits, num_attempts)
        U += H - HT
        r = torch.sum((H - HT) ** 2) / torch.sum(H ** 2)
        s = torch.sum((H - Hp) ** 2) / torch.sum(U ** 2)
        if r < eps and s < eps:
            break
    return H, U
