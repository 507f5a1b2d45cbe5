"""CP-ALS / CP-EPC initialisers (``source/parafac_epc.py:12-82``; tensorly ``parafac``).

The reference delegates to tensorly 0.4.5 ``parafac`` and musco-pytorch 1.0.6
``cp_anc``, neither of which exists offline, so this path is **parity unpinned**
(SURVEY.md §8(c)). ``parafac`` below is a plain fp64 CP-ALS (normalised factors,
relative-error stop) with the reference's call signature; it feeds
``init_factors(init='parafac')``. The EPC rounds (``cp_anc``) of ``parafac_epc``
are the next row of SURVEY.md §8(f) and raise ``NotImplementedError`` until then,
except ``epc_rounds=0``, which returns the CP-ALS factors in the reference's
return layout ``(lmbda, Us)`` with the original mode order.
"""
from __future__ import annotations

from typing import List, Tuple

import torch


def _khatri_rao(mats: List[torch.Tensor]) -> torch.Tensor:
    out = mats[0]
    for m in mats[1:]:
        out = (out[:, None, :] * m[None, :, :]).reshape(-1, out.shape[1])
    return out


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
            others = [fs[k] for k in range(n) if k != m]
            G = torch.ones(rank, rank, dtype=torch.float64, device=X.device)
            for o in others:
                G = G * (o.T @ o)
            unf = torch.moveaxis(X, m, 0).reshape(X.shape[m], -1)
            F = unf @ _khatri_rao(others)
            fs[m] = torch.linalg.solve(G, F.T).T
        rec = torch.einsum(','.join(f'{chr(105 + k)}r' for k in range(n)) + '->' + ''.join(chr(105 + k) for k in range(n)),
                           *fs)
        err = (torch.linalg.norm(X - rec) / norm_x).item()
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


def parafac_epc(tensor, rank, als_maxiter=5000, als_tol=1e-5, num_threads=4, init="random", epc_maxiter=5000,
                epc_rounds=50, epc_tol=1e-5, stop_tol=1e-4, ratio_tol=1e-3, ratio_max_iters=10):
    """source/parafac_epc.py:12-82 signature. CP-ALS is implemented; EPC rounds are not yet."""
    X = torch.as_tensor(tensor, dtype=torch.float64)
    order = sorted(range(X.dim()), key=lambda m: X.shape[m])
    Y = X.permute(*order)
    lmbda, fs = parafac(Y, rank, init=init, tol=als_tol, n_iter_max=als_maxiter, normalize_factors=True)
    if epc_rounds > 0:
        raise NotImplementedError("parafac_epc: EPC rounds (musco cp_anc) are SURVEY §8(f) row 2, not built yet; "
                                  "pass epc_rounds=0 for the CP-ALS factors")
    inv = [0] * len(order)
    for pos, m in enumerate(order):
        inv[m] = pos
    return lmbda, [fs[inv[m]] for m in range(X.dim())]
