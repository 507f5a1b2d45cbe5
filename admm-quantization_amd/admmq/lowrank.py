"""Quant + low-rank ADMM on the MI355X (``scripts/factorize_lowrank.py``).

W is split as W ≈ W_q + W_r, W_q on a ``bits``-bit grid and W_r of rank ``rank``, by
alternating two ADMM solves (``:156-170``), each ``admm_iteration(H, U, W, H2, proj_func,
rho, max_iter, eps)`` (``:85-101``) with the other part held fixed.

* The updates around the projection run as two fused HIP streams (C-ABI
  ``admmq_lowrank_pre`` / ``admmq_lowrank_post``, bit-exact float32 op order) and the
  ``r < eps and s < eps`` break is tested on the device: iterations are queued without a
  host round trip each (the reference syncs every iteration); the loop polls the flag
  every ``poll`` iterations to stop queueing early.
* The quantization projection is the HIP quantizer (``admmq.quantize_tensor``).
* The rank projection is ``KrylovProjector`` by default (warm-started block Krylov in
  float64 on the hand-written panel kernels, stops at a residual bound: agrees with the
  exact truncation to ~1e-4 also on the flat spectra of the loop's iterates),
  ``project_rank`` (exact truncated SVD through the library, the reference's semantics;
  ``projection="svd"``) or ``SubspaceProjector`` (warm-started subspace iteration:
  cheaper, but it stalls on flat spectra - kept for comparison).
"""
from __future__ import annotations

import argparse
import ctypes
import os
import time
from functools import partial
from typing import Callable, List, Optional

import torch

from . import _lib, panel
from .quantization import quantize_tensor


def project_rank(H: torch.Tensor, rank: int) -> torch.Tensor:
    """``U[:, :rank] @ diag(S[:rank]) @ Vt[:rank]`` of ``torch.linalg.svd(H)`` (:80-82)."""
    U, S, Vt = torch.linalg.svd(H, full_matrices=False)
    return U[:, :rank] @ torch.diag(S[:rank]) @ Vt[:rank]


class SubspaceProjector:
    """Rank-``rank`` truncation by block subspace iteration, warm-started from the previous
    call's subspace (consecutive ADMM iterates differ little). Each sweep runs
    Q <- orth(X X^T Q) (thin GEMMs on the device) and the small SVD of Q^T X; it stops
    when the top-``rank`` left singular subspace moves by less than ``tol``
    (sin-theta distance sqrt(rank - ||U_prev^T U||_F^2)), then projects.
    ``oversample`` extra columns speed up convergence of the last wanted triplet."""

    def __init__(self, rank: int, oversample: int = 8, tol: float = 3e-6, max_sweeps: int = 100, seed: int = 0):
        self.rank, self.k = rank, rank + oversample
        self.tol, self.max_sweeps, self.seed = tol, max_sweeps, seed
        self.Q: Optional[torch.Tensor] = None
        self.sweeps: List[int] = []

    def __call__(self, X: torch.Tensor) -> torch.Tensor:
        m, n = X.shape
        k = min(self.k, m, n)
        r = min(self.rank, k)
        if self.Q is None or self.Q.shape != (m, k):
            g = torch.Generator().manual_seed(self.seed)
            self.Q = torch.linalg.qr(X @ torch.randn(n, k, generator=g).to(X.device))[0]
        Q = self.Q
        Ur_prev = None
        sweeps = 0
        for sweeps in range(1, self.max_sweeps + 1):
            Q = torch.linalg.qr(X @ (X.T @ Q))[0]
            Ub, S, Vt = torch.linalg.svd(Q.T @ X, full_matrices=False)
            Ur = Q @ Ub[:, :r]
            if Ur_prev is not None:
                c = float(torch.sum((Ur_prev.T @ Ur) ** 2))
                if max(r - c, 0.0) ** 0.5 < self.tol:
                    break
            Ur_prev = Ur
        self.Q = Q
        self.sweeps.append(sweeps)
        return Ur @ torch.diag(S[:r]) @ Vt[:r]


def _chol_step(Z: torch.Tensor, G: torch.Tensor) -> torch.Tensor:
    """``Z L^{-T}`` for ``G = L L^T`` (one Cholesky-QR pass: Q = Z R^{-1}, R = L^T)."""
    L = torch.linalg.cholesky_ex(G)[0]
    return torch.linalg.solve_triangular(L, Z.T, upper=False).T.contiguous()


def orthonormalize(Z: torch.Tensor) -> torch.Tensor:
    """An orthonormal basis of span(Z) (m x k, float64) by shifted Cholesky QR followed by
    two plain passes (sCholQR3, Fukaya et al. 2020): three k x k Gram products, Cholesky
    factors and triangular solves instead of a Householder QR's O(k) launch-bound reflector
    steps; orthogonal to ~1e-15 for cond(Z) up to ~1e15. The basis differs from the QR's by a
    k x k rotation (the Krylov subspace, hence the projection, does not). No host sync: a
    failure shows as a non-orthonormal K at the next Rayleigh-Ritz check, which repairs it."""
    m, k = Z.shape
    eye = torch.eye(k, dtype=Z.dtype, device=Z.device)
    G = panel.gram(Z, Z)
    shift = 11.0 * (m * k + k * (k + 1)) * 2.0 ** -53 * torch.trace(G)
    Q = _chol_step(Z, G + shift * eye)
    for _ in range(2):
        Q = _chol_step(Q, panel.gram(Q, Q))
    return Q


class KrylovProjector:
    """Rank-``rank`` truncation that matches the exact SVD truncation of
    ``project_rank`` (``scripts/factorize_lowrank.py:80-82``) to ``tol`` on the loop's own
    iterates, including the flat spectra of the low-rank ADMM (sigma_r / sigma_{r+1} ~
    1 + 1e-3 for a 4096 x 4096 noise-like target), where plain subspace iteration stalls.

    Block Krylov (randomized block Lanczos, full re-orthogonalization) in float64 on the
    device: K = [Q, (X X^T) Q, (X X^T)^2 Q, ...] with blocks of ``block`` columns, warm-started
    from the previous call's Ritz vectors; every ``check_every`` blocks a Rayleigh-Ritz
    step (eigh of B B^T, B = K^T X) gives the top-``rank`` triplets (sigma_i, u_i, v_i with
    X^T u_i = sigma_i v_i exactly) and the residuals ||X v_i - sigma_i u_i|| / sigma_1; it
    stops when the largest is <= ``tol`` (the truncation then agrees with the exact one to
    about 2 ``tol`` relative: measured on flat spectra, tools/lowrank_bench.py reports it).
    Every pass over X is a hand-written panel kernel (``admmq.panel``: X^T Q, X Y and the
    final U S V^T, X read as float32 and widened in registers); a new block is
    orthonormalized by Cholesky QR (``orthonormalize``); the re-orthogonalization and the
    small eigenproblem are float64 library calls on panels. Each check also measures
    ||K^T K - I|| (same host sync as the residual) and, past ``ortho_tol``, rebuilds K by a
    Householder QR and repeats the check."""

    def __init__(self, rank: int, block: int = 32, tol: float = 2e-5, check_every: int = 4, max_blocks: int = 64,
                 seed: int = 0, ortho_tol: float = 1e-9):
        self.rank, self.block, self.tol = rank, block, tol
        self.check_every, self.max_blocks, self.seed = check_every, max_blocks, seed
        self.ortho_tol = ortho_tol
        self.Q: Optional[torch.Tensor] = None
        self.blocks: List[int] = []
        self.residuals: List[float] = []
        self.repairs = 0

    def __call__(self, X: torch.Tensor) -> torch.Tensor:
        m, n = X.shape
        r = min(self.rank, m, n)
        # blocks at least `rank` wide: the first Rayleigh-Ritz check then already has r Ritz
        # pairs (a narrower K would index past its eigenpairs and wrap to the top ones)
        k = min(max(self.block, r), m, n)
        Xf = X.float().contiguous()
        if self.Q is None or self.Q.shape != (m, k):
            g = torch.Generator().manual_seed(self.seed)
            self.Q = orthonormalize(panel.xy(Xf, torch.randn(n, k, generator=g, dtype=torch.float64).to(X.device)))
        blocks = [self.Q]
        K = self.Q
        Q = self.Q
        res = float("inf")
        nb = 1
        recheck = False
        while True:
            if recheck or nb >= self.max_blocks or K.shape[1] + k > min(m, n):
                do_check = True
            else:
                Z = panel.xy(Xf, panel.xtq(Xf, Q))             # X (X^T Q)
                for _ in range(2):   # full re-orthogonalization against every block so far
                    Z = Z - K @ panel.gram(K, Z)
                Q = orthonormalize(Z)
                blocks.append(Q)
                K = torch.cat(blocks, 1)
                nb += 1
                do_check = nb % self.check_every == 0
            if not do_check:
                continue
            recheck = False
            Bt = panel.xtq(Xf, K)                              # B^T = X^T K, n x (nb k)
            evals, evecs = torch.linalg.eigh(panel.gram(Bt, Bt))   # B B^T, ascending
            idx = torch.arange(evals.shape[0] - 1, evals.shape[0] - 1 - k, -1, device=X.device)   # k <= K's columns
            S = torch.sqrt(torch.clamp(evals[idx], min=0.0))
            Ub = evecs[:, idx]
            U = K @ Ub[:, :r]
            V = (Bt @ Ub[:, :r]) / S[:r]
            res_t = torch.max(torch.linalg.norm(panel.xy(Xf, V) - U * S[:r], dim=0)) / S[0]
            orth_t = (panel.gram(K, K) - torch.eye(K.shape[1], dtype=K.dtype, device=K.device)).abs().max()
            res, orth = torch.stack([res_t, orth_t]).tolist()   # one host sync for both
            if not orth <= self.ortho_tol:   # (NaN included) a block's Cholesky QR failed: rebuild K
                K = torch.linalg.qr(K)[0]
                blocks = [K]
                Q = K[:, -k:]
                self.repairs += 1
                recheck = True
                continue
            if res <= self.tol or nb >= self.max_blocks or K.shape[1] + k > min(m, n):
                self.Q = orthonormalize(K @ Ub[:, :k])   # warm start: the leading Ritz vectors
                self.blocks.append(nb)
                self.residuals.append(res)
                if r <= 32:   # the panel kernel's register tile
                    out = panel.outer((U * S[:r]).contiguous(), V.contiguous())
                    return out if X.dtype == torch.float32 else out.to(X.dtype)
                return ((U * S[:r]) @ V.T).to(X.dtype)


def _is_device_quantizer(f) -> bool:
    return isinstance(f, partial) and f.func is quantize_tensor


def admm_iteration(H: torch.Tensor, U: torch.Tensor, W: torch.Tensor, H2: torch.Tensor,
                   proj_func: Callable[[torch.Tensor], torch.Tensor], rho: float = 1.0, max_iter: int = 50,
                   eps: float = 1e-8, poll: Optional[int] = None, return_iters: bool = False):
    """scripts/factorize_lowrank.py:85-101. Returns (H, U); U is updated in place and
    returned (as in the reference); the caller's H is not written.

    The break flag is read before an iteration's projection every ``poll``
    iterations. Default: 8 for the HIP quantizer (queued without a host round trip;
    an iteration queued after the break is a device no-op), 1 for any other
    projection (an SVD synchronises anyway, and a projection of a stale iterate
    after the break would cost a full SVD)."""
    if poll is None:
        poll = 8 if _is_device_quantizer(proj_func) else 1
    for t in (H, U, W, H2):
        _lib.require_device(t)
    if not (H.shape == U.shape == W.shape == H2.shape):
        raise ValueError("admmq.lowrank: H, U, W, H2 must have one shape")
    lib = _lib.load()
    dev = H.device
    s = _lib.stream_handle(dev)
    n = H.numel()
    Hc = H.contiguous().clone()
    Uc = U if U.is_contiguous() else U.contiguous()
    Wc, H2c = W.contiguous(), H2.contiguous()
    Hb, X = torch.empty_like(Hc), torch.empty_like(Hc)
    ws = _lib.workspace(lib.admmq_lowrank_workspace_size(n), dev)
    wsp, wsn = _lib.ptr(ws), ws.numel()
    _lib.check(lib.admmq_lowrank_reset(wsp, wsn, s), "lowrank_reset")
    for j in range(1, max_iter):
        if poll and j > 1 and (j - 1) % poll == 0 and int(ws[:4].view(torch.int32)[0]):
            break
        _lib.check(lib.admmq_lowrank_pre(_lib.ptr(Hc), _lib.ptr(Uc), _lib.ptr(Wc), _lib.ptr(H2c), _lib.ptr(Hb),
                                         _lib.ptr(X), n, ctypes.c_float(rho), wsp, wsn, s), "lowrank_pre")
        Hn = proj_func(X).contiguous()
        if Hn.shape != Hc.shape or Hn.dtype != torch.float32 or Hn.device != dev:
            raise ValueError("admmq.lowrank: proj_func must return a float32 tensor of X's shape on X's device")
        _lib.check(lib.admmq_lowrank_post(_lib.ptr(Hn), _lib.ptr(Hb), _lib.ptr(Hc), _lib.ptr(Uc), n,
                                          ctypes.c_float(eps), wsp, wsn, s), "lowrank_post")
    if Uc is not U:
        U.copy_(Uc)
    iters = int(ws[:12].view(torch.int32)[2])
    return (Hc, U, iters) if return_iters else (Hc, U)


def factorize_lowrank(W: torch.Tensor, bits: int, rank: int, qscheme: str = "tensor_minmax", max_iter: int = 100,
                      inner_iter: int = 50, rho: float = 1.0, seed: int = 42, projection: str = "krylov",
                      log_every: int = 10, logger=None):
    """The alternating loop of scripts/factorize_lowrank.py:156-170 (init 'random').
    Returns (W_q, W_r, rel_history). Random starts come from the CPU generator (seeded).

    ``projection`` picks the rank projection (``:80-82``): ``"krylov"`` (default) is the
    device block-Krylov projector on the hand-written fp64-MFMA panel kernels (DESIGN.md
    §2.18; pinned to the reference's own trajectory band F10); ``"svd"`` is the exact
    library SVD truncation (``project_rank``, the reference's arithmetic) for callers that
    want it explicitly; ``"subspace"`` the cheaper subspace iteration (comparison only)."""
    _lib.require_device(W)
    dev = W.device
    g = torch.Generator().manual_seed(seed)
    quant = partial(quantize_tensor, qscheme=qscheme, bits=bits)
    proj = (partial(project_rank, rank=rank) if projection == "svd" else
            KrylovProjector(rank, seed=seed) if projection == "krylov" else SubspaceProjector(rank, seed=seed))
    W_q = torch.randn(*W.shape, generator=g).to(dev)
    U_q = torch.zeros_like(W_q)
    W_r = proj(torch.randn(*W.shape, generator=g).to(dev))
    U_r = torch.zeros_like(W_r)
    hist = []
    nw = torch.linalg.norm(W)
    for i in range(max_iter):
        W_q, U_q = admm_iteration(W_q, U_q, W, W_r, quant, rho=rho, max_iter=inner_iter)
        W_r, U_r = admm_iteration(W_r, U_r, W, W_q, proj, rho=rho, max_iter=inner_iter)
        rel = float(torch.linalg.norm(W - W_r - W_q) / nw)
        if logger and i % log_every == 0:
            logger(f"Diff between W and (W_q + W_r) rel: {rel:.4f}")
        if hist and hist[-1] < rel - 1:
            hist.append(rel)
            break
        hist.append(rel)
    return W_q, W_r, hist


def main(argv=None):
    """CLI of scripts/factorize_lowrank.py (same flags). Pretrained weights cannot be
    downloaded here: ``--weights`` loads a state_dict (weights_only), else the layer is
    a seeded synthetic Llama-7B weight of the same shape (admmq.synthetic)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--model-id", type=str, default="huggyllama/llama-7b")
    ap.add_argument("--cache-dir", type=str, default=None)
    ap.add_argument("--output-dir", type=str, default=".")
    ap.add_argument("--with-wandb", action="store_true")
    ap.add_argument("--layer", type=str, default="model.layers.0.self_attn.q_proj")
    ap.add_argument("--max-iter", required=True, type=int)
    ap.add_argument("--bits", required=True, type=int)
    ap.add_argument("--rank", required=True, type=int)
    ap.add_argument("--qscheme", type=str, default="tensor_minmax")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--weights", type=str, default=None)
    ap.add_argument("--projection", choices=["svd", "krylov", "subspace"], default="krylov",
                    help="rank projection: device block-Krylov on the panel kernels (default) or the exact library "
                         "SVD truncation of the reference (svd)")
    a = ap.parse_args(argv)
    if not torch.cuda.is_available():
        raise RuntimeError("admmq.lowrank needs a ROCm GPU")
    dev = torch.device("cuda:0")
    if a.weights:
        W = torch.load(a.weights, map_location="cpu", weights_only=True)[f"{a.layer}.weight"].float()
    else:
        from . import synthetic
        short = a.layer.split("layers.0.")[-1]
        specs = {s.name: (i, s) for i, s in enumerate(synthetic.llama_layers())}
        i, spec = specs.get(short, (0, synthetic.llama_layers()[0]))
        W = torch.from_numpy(synthetic.layer_weight(spec, i))
    W = W.to(dev)
    t0 = time.time()
    W_q, W_r, hist = factorize_lowrank(W, a.bits, a.rank, a.qscheme, a.max_iter, seed=a.seed,
                                       projection=a.projection, logger=print)
    print(f"done in {time.time() - t0:.1f}s, rel {hist[-1]:.4f}")
    os.makedirs(a.output_dir, exist_ok=True)
    rel = hist[-1]
    torch.save(W_q.cpu(), os.path.join(a.output_dir, f'{a.layer}_{a.bits}_{a.rank}_{rel:.3f}_Q.pt'))
    torch.save(W_r.cpu(), os.path.join(a.output_dir, f'{a.layer}_{a.bits}_{a.rank}_{rel:.3f}_R.pt'))
    return W_q, W_r, hist


if __name__ == "__main__":
    main()
