"""ORACLE — test infrastructure only. CPU restatement of the reference ADMM path.

Restates (numpy/scipy, float32 arithmetic like the reference):
  * ``squared_relative_diff``      source/admm.py:14-15
  * ``unfold``                     source/utils.py:60-74
  * ``admm_iteration``             source/admm.py:51-67 (Cholesky of G+ρI, then
    max_iter-1 iterations of {cholesky_solve, quantize, dual update, residuals})
  * the ALS drivers                scripts/factorize.py:207-266 (3-way), 269-310 (2-way)

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may use this module. Pinned against reference outputs in tests/golden/f2_admm.npz
(few-step ADMM), f3_als.npz (short ALS) and f4_band.json (20×20 ALS objective).

Known, documented deviations (float32 LAPACK differs from torch's): the Cholesky
factor/solve come from scipy's LAPACK (spotrf/spotrs) instead of torch's; residual
sums are accumulated in float64. SURVEY.md §0 shows the trajectory is chaotic at
the 1-ulp level, so parity is stated per horizon (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla

from . import quant_oracle as qo

F32 = np.float32


def squared_relative_diff(X, Y) -> float:
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    return float(np.sqrt(np.sum((X - Y) ** 2) / np.sum(X ** 2)))


def unfold(tensor: np.ndarray, mode: int) -> np.ndarray:
    return np.reshape(np.moveaxis(tensor, mode, 0), (tensor.shape[mode], -1))


def rho_of(G: np.ndarray) -> np.float32:
    """ρ = trace(G)/R (source/admm.py:53); torch-CPU trace accumulates in double."""
    R = G.shape[0]
    tr = F32(np.sum(np.diag(G).astype(np.float64)))
    return F32(tr / F32(R))


def shifted_gram(G: np.ndarray, rho: np.float32) -> np.ndarray:
    A = np.array(G, dtype=F32, copy=True)
    idx = np.arange(A.shape[0])
    A[idx, idx] = (A[idx, idx] + rho).astype(F32)
    return A


def admm_iteration(H, U, F, G, max_iter, eps, bits, qscheme, num_attempts=200, solver="cholesky",
                   return_info=False):
    """source/admm.py:51-67. Returns (H, U) with U a NEW array (callers that need the
    reference's in-place update copy it back). ``solver='inverse'`` uses the
    explicit fp64 inverse rounded to fp32 (the formulation the HIP path uses)."""
    H = np.asarray(H, dtype=F32)
    U = np.array(U, dtype=F32, copy=True)
    F = np.asarray(F, dtype=F32)
    G = np.asarray(G, dtype=F32)
    rho = rho_of(G)
    A = shifted_gram(G, rho)
    if solver == "cholesky":
        fac = sla.cho_factor(A, lower=True, check_finite=False)
    else:
        Minv = np.linalg.inv(A.astype(np.float64))
        M = ((Minv + Minv.T) * 0.5).astype(F32)
    kw = {"num_attempts": num_attempts} if qscheme == "tensor_mseminmax_symmetric" else {}
    iters = 0
    HT = None
    for _ in range(1, max_iter):
        rhs = (F + (rho * (H + U).astype(F32)).astype(F32)).astype(F32)
        if solver == "cholesky":
            HT = sla.cho_solve(fac, rhs.T, check_finite=False).T.astype(F32)
        else:
            HT = (rhs @ M).astype(F32)
        H_prev = H
        H = qo.quantize_tensor((HT - U).astype(F32), bits, qscheme, **kw)
        U = (U + (H - HT).astype(F32)).astype(F32)
        iters += 1
        r = np.sum(((H - HT).astype(F32).astype(np.float64)) ** 2) / np.sum(H.astype(np.float64) ** 2)
        s = np.sum(((H - H_prev).astype(F32).astype(np.float64)) ** 2) / np.sum(U.astype(np.float64) ** 2)
        if r < eps and s < eps:
            break
    if return_info:
        return H, U, dict(iters=iters, HT=HT, rho=rho)
    return H, U


def gram_mttkrp(W, factors, mode):
    """scripts/factorize.py:215-237 (3-way) / 276-287 (2-way)."""
    W = np.asarray(W, dtype=F32)
    if W.ndim == 3:
        A, B, C = factors
        if mode == 0:
            return ((B.T @ B) * (C.T @ C)).astype(F32), np.einsum('abc,cr,br->ar', W, C, B).astype(F32)
        if mode == 1:
            return ((A.T @ A) * (C.T @ C)).astype(F32), np.einsum('abc,cr,ar->br', W, C, A).astype(F32)
        return ((A.T @ A) * (B.T @ B)).astype(F32), np.einsum('abc,br,ar->cr', W, B, A).astype(F32)
    A, B = factors
    if mode == 0:
        return (B.T @ B).astype(F32), (W @ B).astype(F32)
    return (A.T @ A).astype(F32), (W.T @ A).astype(F32)


def reconstruct(factors):
    if len(factors) == 3:
        return np.einsum('ir,jr,kr->ijk', *factors)
    return factors[0] @ factors[1].T


def als(W, init_factors, max_iter_als, max_iter_admm, bits=4, qscheme="tensor_mseminmax_symmetric",
        eps=1e-8, tol=1e-5, solver="cholesky"):
    """scripts/factorize.py:178-310: ALS over modes, ADMM per mode, re-quantize,
    two reconstruction errors per sweep, the |Δloss|<tol and exploding-error stops."""
    W = np.asarray(W, dtype=F32)
    fs = [np.asarray(f, dtype=F32).copy() for f in init_factors]
    Us = [np.zeros_like(f) for f in fs]
    qf = [None] * len(fs)
    loss, lossq = [], []
    back = 5 if W.ndim == 3 else 10
    for _ in range(max_iter_als):
        for m in range(len(fs)):
            G, F = gram_mttkrp(W, fs, m)
            fs[m], Us[m] = admm_iteration(fs[m], Us[m], F, G, max_iter_admm, eps, bits, qscheme, solver=solver)
            qf[m] = qo.quantize_tensor(fs[m], bits, qscheme)
        loss.append(squared_relative_diff(W, reconstruct(fs)))
        lossq.append(squared_relative_diff(W, reconstruct(qf)))
        if len(loss) > 1 and abs(loss[-2] - loss[-1]) < tol:
            break
        if len(loss) > 10 and loss[-1] - loss[-back] > 1e-3:
            break
    return fs, qf, loss, lossq
