"""CPU oracle of the CP-ALS / CP-EPC initialisers (TEST INFRASTRUCTURE: only tests/ import
this module; the product is ``admmq.parafac_epc``, whose per-mode contractions run on the
fp64 HIP kernels of ``csrc/cp64_kernels.hip``).

The reference (``source/parafac_epc.py:12-82``) delegates to tensorly 0.4.5 ``parafac``
and musco-pytorch 1.0.6 ``cp_anc``, neither of which exists offline, so this restatement
is **parity unpinned** (SURVEY.md §8(c)): it restates the published algorithms in fp64
torch on the CPU and keeps the reference's call signature, control flow and return layout:

* ``parafac``: fp64 CP-ALS (random init, relative-error stop), optional column
  normalisation into ``weights`` (tensorly's ``normalize_factors=True``).
* ``cp_anc``: the error-preserving correction (EPC) of Phan et al., "Stable low-rank
  tensor decomposition for compression of convolutional neural network" (ECCV 2020):
  minimise the intensities ||lambda||^2 subject to ||Y - [[lambda; U]]||_F <= delta, by
  alternating over modes. For mode n, with the other factors column-normalised (their
  norms absorbed into U_n, so ||U_n||_F^2 = ||lambda||^2), the sub-problem
  ``min ||U_n||^2 s.t. ||Y_(n) - U_n Z^T||^2 <= delta^2`` has the closed form
  U_n = F V diag(1 / (s + mu)) V^T (F = Y_(n) Z the MTTKRP, Z^T Z = V diag(s) V^T the
  Hadamard product of the Grams), mu >= 0 the root of the monotone error equation
  ||Y||^2 - sum_j |F v_j|^2 (s_j + 2 mu) / (s_j + mu)^2 = delta^2 (mu = 0 when the
  least-squares error already exceeds delta).
* ``parafac_epc``: the reference's driver (``:12-82``): modes sorted by size, CP-ALS,
  delta = the ALS error, EPC rounds until the intensity norm or the max/min intensity
  ratio settles; factors returned in the original mode order.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch


def _khatri_rao(mats: List[torch.Tensor]) -> torch.Tensor:
    out = mats[0]
    for m in mats[1:]:
        out = (out[:, None, :] * m[None, :, :]).reshape(-1, out.shape[1])
    return out


def _unfold(X: torch.Tensor, mode: int) -> torch.Tensor:
    return torch.moveaxis(X, mode, 0).reshape(X.shape[mode], -1)


def _mttkrp_gram(X: torch.Tensor, fs: Sequence[torch.Tensor], mode: int):
    others = [fs[k] for k in range(len(fs)) if k != mode]
    G = torch.ones(fs[0].shape[1], fs[0].shape[1], dtype=X.dtype, device=X.device)
    for o in others:
        G = G * (o.T @ o)
    return _unfold(X, mode) @ _khatri_rao(others), G


def _reconstruct(weights: Optional[torch.Tensor], fs: Sequence[torch.Tensor]) -> torch.Tensor:
    A = fs[0] * weights if weights is not None else fs[0]
    return (A @ _khatri_rao(list(fs[1:])).T).reshape(*[f.shape[0] for f in fs])


def parafac(tensor: torch.Tensor, rank: int, init: str = "random", random_state=None, tol: float = 1e-8,
            n_iter_max: int = 100, normalize_factors: bool = False) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """fp64 CP-ALS on the tensor's device; returns (weights, factors)."""
    X = tensor.to(torch.float64)
    n = X.dim()
    gen = torch.Generator(device="cpu")
    gen.manual_seed(0 if random_state is None else int(random_state))
    if init != "random":
        raise NotImplementedError(f"parafac init={init!r}")
    fs = [torch.rand(X.shape[m], rank, generator=gen, dtype=torch.float64).to(X.device) for m in range(n)]
    norm_x = torch.linalg.norm(X)
    prev = None
    for _ in range(n_iter_max):
        for m in range(n):
            F, G = _mttkrp_gram(X, fs, m)
            fs[m] = torch.linalg.solve(G, F.T).T
        err = (torch.linalg.norm(X - _reconstruct(None, fs)) / norm_x).item()
        if prev is not None and abs(prev - err) < tol:
            break
        prev = err
    weights = torch.ones(rank, dtype=torch.float64, device=X.device)
    if normalize_factors:
        for m in range(n):
            nrm = torch.linalg.norm(fs[m], dim=0)
            weights = weights * nrm
            fs[m] = fs[m] / nrm
    return weights, fs


def _solve_mu(c: torch.Tensor, s: torch.Tensor, normY2: float, delta2: float) -> float:
    """Root mu >= 0 of normY2 - sum c (s + 2 mu) / (s + mu)^2 = delta2 (increasing in mu)."""
    def err(mu: float) -> float:
        return normY2 - float(torch.sum(c * (s + 2 * mu) / (s + mu) ** 2))
    if err(0.0) >= delta2:
        return 0.0
    hi = max(float(s.max()), 1e-300)
    while err(hi) < delta2 and hi < 1e300:
        hi *= 2.0
    lo = 0.0
    for _ in range(200):   # bisection to fp64 resolution of the bracket
        mid = 0.5 * (lo + hi)
        if mid <= lo or mid >= hi:
            break
        if err(mid) < delta2:
            lo = mid
        else:
            hi = mid
    return lo   # the feasible end of the bracket: err(lo) < delta2


def cp_anc(tensor: torch.Tensor, rank: int, delta: float, weights: Optional[torch.Tensor] = None,
           factors: Optional[Sequence[torch.Tensor]] = None, maxiter: int = 5000, tol: float = 1e-5
           ) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """EPC correction (see the module docstring). Returns (weights, column-normalised
    factors) with ||Y - [[weights; factors]]|| = delta (or the LS error if larger)."""
    Y = tensor.to(torch.float64)
    n = Y.dim()
    fs = [f.to(device=Y.device, dtype=torch.float64).clone() for f in factors]
    if weights is not None:
        fs[-1] = fs[-1] * weights.to(fs[-1])
    normY2 = float(torch.sum(Y * Y))
    delta2 = float(delta) ** 2
    lam_prev = None
    lam = torch.ones(rank, dtype=torch.float64, device=Y.device)
    for _ in range(max(int(maxiter), 1)):
        for m in range(n):
            # normalise the other factors, moving their column norms into factor m
            for k in range(n):
                if k != m:
                    nrm = torch.linalg.norm(fs[k], dim=0).clamp_min(1e-300)
                    fs[k] = fs[k] / nrm
                    fs[m] = fs[m] * nrm
            F, G = _mttkrp_gram(Y, fs, m)
            s, V = torch.linalg.eigh(G)
            s = s.clamp_min(0.0)
            Ft = F @ V
            mu = _solve_mu(torch.sum(Ft * Ft, dim=0), s, normY2, delta2)
            fs[m] = (Ft / (s + mu).clamp_min(1e-300)) @ V.T
        lam = torch.linalg.norm(fs[n - 1], dim=0)
        lnorm = float(torch.linalg.norm(lam))
        if lam_prev is not None and abs(lam_prev - lnorm) < tol * lam_prev:
            break
        lam_prev = lnorm
    # final normalisation: every factor unit-norm columns, intensities in the weights
    weights = torch.ones(rank, dtype=torch.float64, device=Y.device)
    for m in range(n):
        nrm = torch.linalg.norm(fs[m], dim=0).clamp_min(1e-300)
        weights = weights * nrm
        fs[m] = fs[m] / nrm
    return weights, fs


def parafac_epc(tensor, rank, als_maxiter=5000, als_tol=1e-5, num_threads=4, init="random", epc_maxiter=5000,
                epc_rounds=50, epc_tol=1e-5, stop_tol=1e-4, ratio_tol=1e-3, ratio_max_iters=10):
    """source/parafac_epc.py:12-82 -> (lmbda, Us), Us in the tensor's mode order.

    ``num_threads`` is accepted for signature compatibility; unlike the reference it does
    not change torch's global thread count (source/parafac_epc.py:33)."""
    X = torch.as_tensor(tensor).to(torch.float64)
    order = sorted(range(X.dim()), key=lambda m: X.shape[m])
    Y = X.permute(*order)
    lmbda, fs = parafac(Y, rank, init=init, tol=als_tol, n_iter_max=als_maxiter, normalize_factors=True)
    delta = float(torch.linalg.norm(Y - _reconstruct(lmbda, fs)))
    lambda_norm_prev = float(torch.linalg.norm(lmbda))
    alpha_prev = float(lmbda.max() / lmbda.min())
    stopflag = 0
    for _ in range(epc_rounds):
        lmbda, fs = cp_anc(Y, rank, delta, lmbda, fs, maxiter=epc_maxiter, tol=epc_tol)
        lambda_norm = float(torch.linalg.norm(lmbda))
        alpha = float(lmbda.max() / lmbda.min())
        if abs(lambda_norm_prev - lambda_norm) < stop_tol * lambda_norm_prev:
            break
        stopflag = stopflag + 1 if abs(alpha_prev - alpha) < ratio_tol else 0
        lambda_norm_prev, alpha_prev = lambda_norm, alpha
        if stopflag >= ratio_max_iters:
            break
    inv = [0] * len(order)
    for pos, m in enumerate(order):
        inv[m] = pos
    return lmbda, [fs[inv[m]] for m in range(X.dim())]
