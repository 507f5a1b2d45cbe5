"""CP-ALS / CP-EPC initialisers on the MI355X (``source/parafac_epc.py:12-82``; tensorly
``parafac``, musco-pytorch ``cp_anc``).

The reference delegates to tensorly 0.4.5 ``parafac`` and musco-pytorch 1.0.6
``cp_anc``, neither of which exists offline, so this module is **parity unpinned**
(SURVEY.md §8(c)); it restates the published algorithms (the CPU restatement used as
the test oracle is ``oracle/epc_oracle.py``) and keeps the reference's call signature,
control flow and return layout:

* ``parafac``: fp64 CP-ALS (random init, relative-error stop), optional column
  normalisation into ``weights`` (tensorly's ``normalize_factors=True``).
* ``cp_anc``: the error-preserving correction (EPC) of Phan et al. (ECCV 2020): per mode
  the closed form U_n = F V diag(1 / (s + mu)) V^T (F = Y_(n) Z the MTTKRP,
  Z^T Z = V diag(s) V^T the Hadamard product of the Grams, mu >= 0 the root of the
  monotone error equation; see ``oracle/epc_oracle.py`` for the derivation).
* ``parafac_epc``: the reference's driver (``:12-82``): modes sorted by size, CP-ALS,
  delta = the ALS error, EPC rounds until the intensity norm or the max/min intensity
  ratio settles; factors returned in the original mode order.

Device placement: every per-mode MTTKRP and Gram-Hadamard product (the O(I J K R) work)
runs on the fp64 HIP kernels (``als.gram_mttkrp_f64`` -> ``csrc/cp64_kernels.hip``, f64
MFMA with the Khatri-Rao operand formed on the fly); the reconstruction errors use the
CP identity ||Y||^2 - 2 <Y, [[w; U]]> + ||[[w; U]]||^2 on those products (no I x J x K
reconstruction, as tensorly's ``parafac`` does); the R x R solves run on one workgroup with
the matrix in LDS (``panel.spd_solve64`` for the CP-ALS update, ``panel.epc_step64`` for the
EPC update: Cholesky factors of G + mu I and Newton steps on the error equation instead of
an eigendecomposition; ``csrc/epc_kernels.hip``) for R <= 136, torch linear algebra above
that. The stopping scalars stay on the device: the drivers run ``_CHECK_EVERY`` iterations
between host reads, keep each iteration's factors, and on a stop return those of the
iteration the reference would have stopped at (the same iterations and results as a
per-iteration check, without its host synchronisation).
Float64 tensors on the GPU only: a CPU tensor raises (no CPU path).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from .als import gram_mttkrp_f64
from .panel import SPD_SMALL_MAX, colnorm64, epc_mu, epc_step64, spd_solve64

_CHECK_EVERY = 8   # iterations between the host's reads of the device-side stop tests


def _khatri_rao(mats: List[torch.Tensor]) -> torch.Tensor:
    out = mats[0]
    for m in mats[1:]:
        out = (out[:, None, :] * m[None, :, :]).reshape(-1, out.shape[1])
    return out


def _reconstruct(weights: Optional[torch.Tensor], fs: Sequence[torch.Tensor]) -> torch.Tensor:
    """[[weights; fs]] materialised (diagnostics and tests; the driver never builds it)."""
    A = fs[0] * weights if weights is not None else fs[0]
    return (A @ _khatri_rao(list(fs[1:])).T).reshape(*[f.shape[0] for f in fs])


def _on_gpu64(tensor) -> torch.Tensor:
    X = torch.as_tensor(tensor)
    if X.device.type != "cuda":
        raise RuntimeError("admmq.parafac_epc runs on the ROCm GPU: move the tensor to a 'cuda' device "
                           "(there is no CPU path)")
    return X.to(torch.float64)


def _cp_error2(normY2, F_last: torch.Tensor, G_last: torch.Tensor, U_last: torch.Tensor,
               weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """||Y - [[w; U]]||^2 (a 0-dim device tensor: no host synchronisation) from the last
    mode's MTTKRP F and Gram-Hadamard G (of the other factors) and its factor:
    ||Y||^2 - 2 <F, U w> + w^T (G * U^T U) w."""
    Uw = U_last * weights if weights is not None else U_last
    inner = torch.sum(F_last * Uw)
    norm2 = torch.sum(G_last * (Uw.T @ Uw))
    return torch.clamp(normY2 - 2.0 * inner + norm2, min=0.0)


def _als_update(G: torch.Tensor, F: torch.Tensor) -> torch.Tensor:
    """tensorly parafac's factor update U = F G^-1 (G = Hadamard of the other Grams)."""
    if G.shape[0] <= SPD_SMALL_MAX:
        return spd_solve64(G, F)
    return torch.linalg.solve(G, F.T).T


def parafac(tensor: torch.Tensor, rank: int, init: str = "random", random_state=None, tol: float = 1e-8,
            n_iter_max: int = 100, normalize_factors: bool = False) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """fp64 CP-ALS on the GPU; returns (weights, factors)."""
    X = _on_gpu64(tensor).contiguous()
    n = X.dim()
    gen = torch.Generator(device="cpu")
    gen.manual_seed(0 if random_state is None else int(random_state))
    if init != "random":
        raise NotImplementedError(f"parafac init={init!r}")
    fs = [torch.rand(X.shape[m], rank, generator=gen, dtype=torch.float64).to(X.device) for m in range(n)]
    normY2 = torch.sum(X * X)
    norm_x = torch.sqrt(normY2)
    prev = None
    it = 0
    while it < n_iter_max:
        # a chunk of iterations between host reads: every iteration's factors and error kept
        snaps, errs = [], []
        for _ in range(min(_CHECK_EVERY, n_iter_max - it)):
            for m in range(n):
                F, G = gram_mttkrp_f64(X, fs, m)
                fs[m] = _als_update(G, F)
            errs.append(torch.sqrt(_cp_error2(normY2, F, G, fs[n - 1])) / norm_x)   # F, G of the last mode
            snaps.append(list(fs))
        it += len(errs)
        ev = torch.stack(errs).tolist()   # the chunk's one host read
        stop = None
        for k, err in enumerate(ev):
            if prev is not None and abs(prev - err) < tol:
                stop = k
                break
            prev = err
        if stop is not None:
            fs = snaps[stop]
            break
    weights = torch.ones(rank, dtype=torch.float64, device=X.device)
    if normalize_factors:
        for m in range(n):
            nrm = torch.linalg.norm(fs[m], dim=0)
            weights = weights * nrm
            fs[m] = fs[m] / nrm
    return weights, fs


def _epc_update(G: torch.Tensor, F: torch.Tensor, normY2: float, delta2: float, mu: torch.Tensor) -> torch.Tensor:
    """cp_anc's mode update U_n = F (G + mu I)^-1 with mu on the error equation."""
    if G.shape[0] <= SPD_SMALL_MAX:
        return epc_step64(G, F, normY2, delta2, mu)
    s, V = torch.linalg.eigh(G)
    s = s.clamp_min(0.0)
    Ft = F @ V
    mu.copy_(epc_mu(torch.sum(Ft * Ft, dim=0), s, normY2, delta2))   # on the device: no host sync
    return (Ft / (s + mu).clamp_min(1e-300)) @ V.T


def cp_anc(tensor: torch.Tensor, rank: int, delta: float, weights: Optional[torch.Tensor] = None,
           factors: Optional[Sequence[torch.Tensor]] = None, maxiter: int = 5000, tol: float = 1e-5
           ) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """EPC correction (module docstring). Returns (weights, column-normalised factors)
    with ||Y - [[weights; factors]]|| = delta (or the LS error if larger)."""
    Y = _on_gpu64(tensor).contiguous()
    n = Y.dim()
    fs = [f.to(device=Y.device, dtype=torch.float64).clone() for f in factors]
    if weights is not None:
        fs[-1] = fs[-1] * weights.to(fs[-1])
    normY2 = float(torch.sum(Y * Y))
    delta2 = float(delta) ** 2
    mus = [torch.zeros((), dtype=torch.float64, device=Y.device) for _ in range(n)]   # warm starts per mode
    lam_prev = None
    it, total = 0, max(int(maxiter), 1)
    while it < total:
        snaps, lnorms = [], []
        for _ in range(min(_CHECK_EVERY, total - it)):
            for m in range(n):
                # normalise the other factors, one launch for both (moving their column norms
                # into factor m, as cp_anc does, would be dead work here: factor m is recomputed
                # from F and G below before anything reads it)
                o = [k for k in range(n) if k != m]
                a, b = colnorm64(fs[o[0]], fs[o[1]] if len(o) > 1 else None)
                fs[o[0]] = a
                if len(o) > 1:
                    fs[o[1]] = b
                F, G = gram_mttkrp_f64(Y, fs, m)
                fs[m] = _epc_update(G, F, normY2, delta2, mus[m])
            lnorms.append(torch.linalg.norm(torch.linalg.norm(fs[n - 1], dim=0)))
            snaps.append(list(fs))
        it += len(lnorms)
        lv = torch.stack(lnorms).tolist()   # the chunk's one host read
        stop = None
        for k, lnorm in enumerate(lv):
            if lam_prev is not None and abs(lam_prev - lnorm) < tol * lam_prev:
                stop = k
                break
            lam_prev = lnorm
        if stop is not None:
            fs = snaps[stop]
            break
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
    X = _on_gpu64(tensor)
    order = sorted(range(X.dim()), key=lambda m: X.shape[m])
    Y = X.permute(*order).contiguous()
    lmbda, fs = parafac(Y, rank, init=init, tol=als_tol, n_iter_max=als_maxiter, normalize_factors=True)
    last = Y.dim() - 1
    F, G = gram_mttkrp_f64(Y, fs, last)
    delta = float(_cp_error2(torch.sum(Y * Y), F, G, fs[last], lmbda)) ** 0.5
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
