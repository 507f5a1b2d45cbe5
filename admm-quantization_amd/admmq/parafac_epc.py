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
  the closed form U_n = F (G + mu I)^-1 (F = Y_(n) Z the MTTKRP, G = Z^T Z the Hadamard
  product of the Grams, mu >= 0 the root of the monotone error equation; see
  ``oracle/epc_oracle.py`` for the derivation).
* ``parafac_epc``: the reference's driver (``:12-82``): modes sorted by size, CP-ALS,
  delta = the ALS error, EPC rounds until the intensity norm or the max/min intensity
  ratio settles; factors returned in the original mode order.
* ``parafac_epc_many``: the same for several tensors at once (a model's layers; the
  reference runs ``scripts/factorize.py --init parafac-epc`` once per layer), each on its
  own HIP stream, so one layer's latency-bound solves overlap the others'.

Device placement: every per-mode MTTKRP and Gram-Hadamard product (the O(I J K R) work)
runs on the fp64 HIP kernels (``als.gram_mttkrp_f64`` -> ``csrc/cp64_kernels.hip``, f64
MFMA with the Khatri-Rao operand formed on the fly); the reconstruction errors use the
CP identity ||Y||^2 - 2 <Y, [[w; U]]> + ||[[w; U]]||^2 on those products (no I x J x K
reconstruction, as tensorly's ``parafac`` does). The R x R solves are HIP kernels at every
rank, no torch linear algebra (``admmq.panel``):
* R <= 136, one workgroup with the matrix in LDS (``csrc/epc_kernels.hip``): the CP-ALS
  update by a blocked Gauss-Jordan inverse; the EPC update by one Householder reduction of
  G to tridiagonal form and Newton steps of the multiplier on tridiagonal L D L^T
  recurrences;
* larger R (``csrc/solve64.hip``): the blocked fp64 Cholesky of G (+ mu I) and its inverse
  factor spread over the chip, X = (F L^-T) L^-1 on fp64 MFMA; the EPC multiplier search
  runs on the device (one Cholesky per evaluation), the host reading its done flag every
  few evaluations.
A CP-ALS update whose G is not numerically positive definite (its solve reports it) is
redone for the whole chunk with a relative shift of 1e-10 trace(G)/n on the diagonal; an EPC
update that finds no positive definite G + mu I raises ``torch.linalg.LinAlgError``.
The stopping scalars stay on the device: the drivers run ``_CHECK_EVERY`` iterations
between host reads, keep each iteration's factors, and on a stop return those of the
iteration the reference would have stopped at (the same iterations and results as a
per-iteration check, without its host synchronisation). The drivers are generators that
yield a ``torch.cuda.Event`` at every host read (``_drive`` runs one to completion;
``parafac_epc_many`` interleaves several).
Float64 tensors on the GPU only: a CPU tensor raises (no CPU path).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from .als import gram_mttkrp_f64
from .panel import SPD_SMALL_MAX, colnorm64, epc_step64, epc_step64_gen, spd_solve64

_CHECK_EVERY = 8   # iterations between the host's reads of the device-side stop tests
_ALS_SHIFT = 1e-10   # relative diagonal shift of a CP-ALS chunk redone after a non-positive-definite G


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


def _host(*ts: torch.Tensor):
    """Generator step: copies device tensors to (pinned) host memory, yields the event recorded
    after the copies and returns the host tensors once resumed (the event has completed)."""
    hs = [t.to("cpu", non_blocking=True) for t in ts]
    ev = torch.cuda.Event()
    ev.record()
    yield ev
    return hs


def _drive(gen):
    """Runs one of this module's generators to completion on the current stream."""
    try:
        ev = next(gen)
        while True:
            ev.synchronize()
            ev = gen.send(None)
    except StopIteration as stop:
        return stop.value


def _colnorms(U: torch.Tensor) -> torch.Tensor:
    """Column 2-norms (the ||U[:, r]|| of tensorly / musco's normalisations)."""
    return torch.sqrt(torch.sum(U * U, dim=0))


def _norm(v: torch.Tensor) -> torch.Tensor:
    return torch.sqrt(torch.sum(v * v))


def _cp_error2(normY2, F_last: torch.Tensor, G_last: torch.Tensor, U_last: torch.Tensor,
               weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """||Y - [[w; U]]||^2 (a 0-dim device tensor: no host synchronisation) from the last
    mode's MTTKRP F and Gram-Hadamard G (of the other factors) and its factor:
    ||Y||^2 - 2 <F, U w> + w^T (G * U^T U) w."""
    Uw = U_last * weights if weights is not None else U_last
    inner = torch.sum(F_last * Uw)
    norm2 = torch.sum(G_last * (Uw.T @ Uw))
    return torch.clamp(normY2 - 2.0 * inner + norm2, min=0.0)


def _parafac_gen(tensor, rank: int, init: str = "random", random_state=None, tol: float = 1e-8,
                 n_iter_max: int = 100, normalize_factors: bool = False):
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
        start = list(fs)
        steps = min(_CHECK_EVERY, n_iter_max - it)
        for shift in (0.0, _ALS_SHIFT):
            fs = list(start)
            snaps, errs = [], []
            infos = torch.zeros(steps * n, dtype=torch.int32, device=X.device)
            for k in range(steps):
                for m in range(n):
                    F, G = gram_mttkrp_f64(X, fs, m)
                    fs[m] = spd_solve64(G, F, info=infos[k * n + m:k * n + m + 1], rel_shift=shift)
                errs.append(torch.sqrt(_cp_error2(normY2, F, G, fs[n - 1])) / norm_x)   # F, G of the last mode
                snaps.append(list(fs))
            ev, iv = yield from _host(torch.stack(errs), infos)   # the chunk's one host read
            if not bool(iv.any()):
                break
            if shift:
                raise torch.linalg.LinAlgError("admmq.parafac: the CP-ALS normal equations are not positive definite "
                                               "even with a relative diagonal shift of %g" % _ALS_SHIFT)
        it += steps
        stop = None
        for k, err in enumerate(ev.tolist()):
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
            nrm = _colnorms(fs[m])
            weights = weights * nrm
            fs[m] = fs[m] / nrm
    return weights, fs


def parafac(tensor: torch.Tensor, rank: int, init: str = "random", random_state=None, tol: float = 1e-8,
            n_iter_max: int = 100, normalize_factors: bool = False) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """fp64 CP-ALS on the GPU; returns (weights, factors)."""
    return _drive(_parafac_gen(tensor, rank, init, random_state, tol, n_iter_max, normalize_factors))


def _cp_anc_gen(tensor, rank: int, delta: float, weights=None, factors=None, maxiter: int = 5000, tol: float = 1e-5,
                mus=None):
    Y = _on_gpu64(tensor).contiguous()
    n = Y.dim()
    fs = [f.to(device=Y.device, dtype=torch.float64).clone() for f in factors]
    if weights is not None:
        fs[-1] = fs[-1] * weights.to(fs[-1])
    (ny,) = yield from _host(torch.sum(Y * Y))
    normY2 = float(ny)
    delta2 = float(delta) ** 2
    if mus is None:   # the multipliers' warm starts per mode (parafac_epc carries them across its rounds)
        mus = [torch.zeros((), dtype=torch.float64, device=Y.device) for _ in range(n)]
    lam_prev = None
    it, total = 0, max(int(maxiter), 1)
    while it < total:
        snaps, lnorms = [], []
        steps = min(_CHECK_EVERY, total - it)
        infos = torch.zeros(steps * n, dtype=torch.int32, device=Y.device)
        for k in range(steps):
            for m in range(n):
                # normalise the other factors, one launch for both (moving their column norms
                # into factor m, as cp_anc does, would be dead work here: factor m is recomputed
                # from F and G below before anything reads it)
                o = [q for q in range(n) if q != m]
                a, b = colnorm64(fs[o[0]], fs[o[1]] if len(o) > 1 else None)
                fs[o[0]] = a
                if len(o) > 1:
                    fs[o[1]] = b
                F, G = gram_mttkrp_f64(Y, fs, m)
                info = infos[k * n + m:k * n + m + 1]
                if G.shape[0] <= SPD_SMALL_MAX:
                    fs[m] = epc_step64(G, F, normY2, delta2, mus[m], info=info)
                else:
                    fs[m] = yield from epc_step64_gen(G, F, normY2, delta2, mus[m], info=info)
            lnorms.append(_norm(_colnorms(fs[n - 1])))
            snaps.append(list(fs))
        it += steps
        lv, iv = yield from _host(torch.stack(lnorms), infos)   # the chunk's one host read
        if bool(iv.any()):
            raise torch.linalg.LinAlgError("admmq.cp_anc: the EPC update found no positive definite G + mu I "
                                           "(or its multiplier search did not converge)")
        stop = None
        for k, lnorm in enumerate(lv.tolist()):
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
        nrm = _colnorms(fs[m]).clamp_min(1e-300)
        weights = weights * nrm
        fs[m] = fs[m] / nrm
    return weights, fs


def cp_anc(tensor: torch.Tensor, rank: int, delta: float, weights: Optional[torch.Tensor] = None,
           factors: Optional[Sequence[torch.Tensor]] = None, maxiter: int = 5000, tol: float = 1e-5
           ) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """EPC correction (module docstring). Returns (weights, column-normalised factors)
    with ||Y - [[weights; factors]]|| = delta (or the LS error if larger)."""
    return _drive(_cp_anc_gen(tensor, rank, delta, weights, factors, maxiter, tol))


def _parafac_epc_gen(tensor, rank, als_maxiter=5000, als_tol=1e-5, num_threads=4, init="random", epc_maxiter=5000,
                     epc_rounds=50, epc_tol=1e-5, stop_tol=1e-4, ratio_tol=1e-3, ratio_max_iters=10):
    X = _on_gpu64(tensor)
    order = sorted(range(X.dim()), key=lambda m: X.shape[m])
    Y = X.permute(*order).contiguous()
    lmbda, fs = yield from _parafac_gen(Y, rank, init=init, tol=als_tol, n_iter_max=als_maxiter,
                                        normalize_factors=True)
    last = Y.dim() - 1
    F, G = gram_mttkrp_f64(Y, fs, last)
    d2, ln, lmax, lmin = yield from _host(_cp_error2(torch.sum(Y * Y), F, G, fs[last], lmbda),
                                          _norm(lmbda), lmbda.max(), lmbda.min())
    delta = float(d2) ** 0.5
    lambda_norm_prev = float(ln)
    alpha_prev = float(lmax) / float(lmin)
    stopflag = 0
    mus = [torch.zeros((), dtype=torch.float64, device=Y.device) for _ in range(Y.dim())]
    for _ in range(epc_rounds):
        lmbda, fs = yield from _cp_anc_gen(Y, rank, delta, lmbda, fs, maxiter=epc_maxiter, tol=epc_tol, mus=mus)
        ln, lmax, lmin = yield from _host(_norm(lmbda), lmbda.max(), lmbda.min())
        lambda_norm = float(ln)
        alpha = float(lmax) / float(lmin)
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


def parafac_epc(tensor, rank, als_maxiter=5000, als_tol=1e-5, num_threads=4, init="random", epc_maxiter=5000,
                epc_rounds=50, epc_tol=1e-5, stop_tol=1e-4, ratio_tol=1e-3, ratio_max_iters=10):
    """source/parafac_epc.py:12-82 -> (lmbda, Us), Us in the tensor's mode order.

    ``num_threads`` is accepted for signature compatibility; unlike the reference it does
    not change torch's global thread count (source/parafac_epc.py:33)."""
    return _drive(_parafac_epc_gen(tensor, rank, als_maxiter, als_tol, num_threads, init, epc_maxiter, epc_rounds,
                                   epc_tol, stop_tol, ratio_tol, ratio_max_iters))


def _drive_many(gens: Sequence, device: torch.device) -> list:
    """Interleaves generators of this module, each on its own HIP stream (forked from the
    current stream): a generator resumes once the event it yielded has completed, so one
    layer's host reads never hold back another layer's queued work. The current stream
    waits for all of them at the end, and the results are recorded as used on it."""
    main = torch.cuda.current_stream(device)
    streams = [torch.cuda.Stream(device) for _ in gens]
    for s in streams:
        s.wait_stream(main)
    pending = [None] * len(gens)   # the event each generator waits on (None: runnable)
    results = [None] * len(gens)
    active = list(range(len(gens)))
    while active:
        progressed = False
        for i in list(active):
            ev = pending[i]
            if ev is not None and not ev.query():
                continue
            progressed = True
            with torch.cuda.stream(streams[i]):
                try:
                    pending[i] = gens[i].send(None)
                except StopIteration as stop:
                    results[i] = stop.value
                    active.remove(i)
        if not progressed:   # every layer waits on the device: block on the oldest
            pending[active[0]].synchronize()
    for s in streams:
        main.wait_stream(s)
    for lm, us in results:
        for t in [lm, *us]:
            t.record_stream(main)
    return results


def parafac_epc_many(tensors: Sequence[torch.Tensor], ranks: Sequence[int], **kwargs) -> list:
    """``parafac_epc`` for several tensors (e.g. all conv layers of a model) at once: the same
    results as calling it on each (every layer's arithmetic and stop tests are its own), with
    the layers running concurrently on separate HIP streams. Returns [(lmbda, Us)] in order."""
    if len(tensors) != len(ranks):
        raise ValueError("parafac_epc_many: one rank per tensor")
    if not tensors:
        return []
    Xs = [_on_gpu64(t) for t in tensors]
    dev = Xs[0].device
    if any(X.device != dev for X in Xs):
        raise ValueError("parafac_epc_many: all tensors on one device")
    return _drive_many([_parafac_epc_gen(X, int(r), **kwargs) for X, r in zip(Xs, ranks)], dev)
