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


def gram_mttkrp(W: torch.Tensor, factors, mode: int):
    """Per-mode setup of scripts/factorize.py:215-237 (3-way) / :276-287 (2-way), in the
    reference's own torch expressions (the einsum strings are the reference's)."""
    if W.dim() == 3:
        A, B, C = factors
        if mode == 0:
            return B.T @ B * (C.T @ C), torch.einsum('abc,cr,br->ar', W, C, B)
        if mode == 1:
            return A.T @ A * (C.T @ C), torch.einsum('abc,cr,ar->br', W, C, A)
        return A.T @ A * (B.T @ B), torch.einsum('abc,br,ar->cr', W, B, A)
    A, B = factors
    if mode == 0:
        return B.T @ B, W @ B
    return A.T @ A, W.T @ A


def rel_error(W: torch.Tensor, factors) -> float:
    """squared_relative_diff(W, [[factors]]) (source/admm.py:14-15, scripts/factorize.py:246-253)."""
    rec = torch.einsum('ir,jr,kr->ijk', *factors) if W.dim() == 3 else factors[0] @ factors[1].T
    return torch.sqrt(torch.sum((W - rec) ** 2) / torch.sum(W ** 2)).item()

