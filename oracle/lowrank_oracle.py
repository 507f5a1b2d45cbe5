"""ORACLE — test infrastructure only. numpy restatement of the quant + low-rank ADMM of
``scripts/factorize_lowrank.py`` (pinned by tests/golden/f6_lowrank.npz).

  * ``project_rank``      scripts/factorize_lowrank.py:80-82  (SVD truncation)
  * ``admm_iteration``    scripts/factorize_lowrank.py:85-101 (float32, reference op order)

Only ``tests/`` may import this module. Residual sums are accumulated in float64 (the
reference sums float32 on its device); they only steer the ``r < eps and s < eps`` break.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def project_rank(H: np.ndarray, rank: int) -> np.ndarray:
    U, S, Vt = np.linalg.svd(np.asarray(H, F32), full_matrices=False)
    return ((U[:, :rank] * S[:rank]) @ Vt[:rank]).astype(F32)


def admm_iteration(H, U, W, H2, proj_func, rho=1.0, max_iter=50, eps=1e-8):
    """Returns (H, U, iterations run). U is a new array (the reference mutates in place)."""
    H = np.asarray(H, F32).copy()
    U = np.asarray(U, F32).copy()
    W = np.asarray(W, F32)
    H2 = np.asarray(H2, F32)
    r32, den = F32(rho), F32(1.0 + rho)
    it = 0
    for _ in range(1, max_iter):
        Hb = (((r32 * (H + U)).astype(F32) + W).astype(F32) - H2).astype(F32) / den
        Hb = Hb.astype(F32)
        Hp = H
        H = np.asarray(proj_func((Hb - U).astype(F32)), F32)
        U = (U + (H - Hb).astype(F32)).astype(F32)
        it += 1
        d = (H - Hb).astype(np.float64)
        dp = (H - Hp).astype(np.float64)
        r = np.sum(d * d) / np.sum(H.astype(np.float64) ** 2)
        s = np.sum(dp * dp) / np.sum(U.astype(np.float64) ** 2)
        if r < eps and s < eps:
            break
    return H, U, it
