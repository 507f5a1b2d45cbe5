"""Drop-in ADMM factor solver (``source/admm.py``) on the MI355X.

``admm_iteration(H, U, F, G, max_iter, eps, bits, qscheme)`` keeps the reference's
signature (positional order as called at ``scripts/factorize.py:218-221``) and
conventions:

* returns ``(H_new, U)``: a new H tensor, and the caller's ``U`` object updated in
  place (``source/admm.py:60``); the caller's ``H``/``F``/``G`` are not written;
* ``max_iter - 1`` inner iterations (``range(1, max_iter)``), each ending with the
  ``r < eps and s < eps`` early exit (``:62-65``); ``max_iter <= 1`` returns the
  input ``H`` object unchanged;
* a non-SPD ``G + rho I`` raises ``torch.linalg.LinAlgError`` before anything is
  modified (``:54``); unknown schemes raise like ``quantize_tensor``.

What differs by design: the Cholesky factor + per-iteration
``cholesky_solve`` are replaced by one fp64 blocked inverse per call and one
fp32-MFMA GEMM per iteration, and the whole loop is a device-side launch
sequence; the call synchronises once at its end (to check the fault column).

``admm_iteration_batched`` runs many independent (layer, mode) problems in the
same launches; it is what the ALS driver and the benchmark use.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from .quantization import _scheme_code
from .utils import unfold

__all__ = ["admm_iteration", "admm_iteration_batched", "init_factors", "init_factors_many", "squared_relative_diff"]


def squared_relative_diff(X: torch.Tensor, Y: torch.Tensor) -> float:
    """source/admm.py:14-15: sqrt(sum((X-Y)^2) / sum(X^2)) (a relative Frobenius error)."""
    return torch.sqrt(torch.sum((X - Y) ** 2) / torch.sum(X ** 2)).item()


def init_factors(tensor: torch.Tensor, rank: int, init: str = "random", device=None, seed=None) -> List[torch.Tensor]:
    """source/admm.py:21-48.

    ``random`` draws ``randn(I_n, rank)`` per mode from a CPU ``torch.Generator``
    seeded with ``seed`` and moves the factors to ``device`` - identical numbers to
    the reference run on CPU (the reference on a GPU would use the device generator,
    whose stream is backend-specific). ``svd`` uses ``torch.linalg.svd`` of the
    mode unfoldings (init only). ``parafac``/``parafac-epc`` call :mod:`admmq.parafac_epc`.
    """
    gen = torch.Generator(device="cpu")
    gen.manual_seed(seed)
    dev = torch.device(device) if device is not None else tensor.device
    factors = []
    if init == "random":
        for mode in range(tensor.ndim):
            factors.append(torch.randn(tensor.shape[mode], rank, generator=gen).to(dev))
    elif init == "svd":
        for mode in range(tensor.ndim):
            Uu, _, _ = torch.linalg.svd(unfold(tensor, mode), full_matrices=False)
            if tensor.shape[mode] < rank:
                rnd = torch.randn(Uu.shape[0], rank - tensor.shape[mode], generator=gen).to(Uu.device)
                Uu = torch.cat((Uu, rnd), dim=1)
            factors.append(Uu[:, :rank].to(dev))
    elif init in ("parafac", "parafac-epc"):
        from .parafac_epc import parafac, parafac_epc
        X = tensor.to(dev)   # fp64 HIP contractions on the device (admmq.parafac_epc)
        if init == "parafac":
            _, factors = parafac(X, rank=rank, init="random", random_state=seed, tol=1e-5, n_iter_max=100)
        else:
            _, factors = parafac_epc(X, rank=rank, init="random", als_maxiter=50, epc_maxiter=50)
        factors = [f.to(device=dev, dtype=torch.float32) for f in factors]
    else:
        raise NotImplementedError(init)
    return factors


def init_factors_many(tensors: Sequence[torch.Tensor], ranks: Sequence[int], init: str = "random", device=None,
                      seed=None) -> List[List[torch.Tensor]]:
    """``init_factors`` for every layer of a model (the reference runs scripts/factorize.py once
    per layer, each calling source/admm.py:21-48): the same factors as one call per layer. With
    ``parafac-epc`` the layers' initialisers run concurrently, one HIP stream each
    (``admmq.parafac_epc.parafac_epc_many``): a model's initialisation then takes about as long
    as its slowest layers instead of the sum."""
    if len(tensors) != len(ranks):
        raise ValueError("init_factors_many: one rank per tensor")
    if init != "parafac-epc" or not tensors:
        return [init_factors(t, rank=r, init=init, device=device, seed=seed) for t, r in zip(tensors, ranks)]
    from .parafac_epc import parafac_epc_many
    dev = torch.device(device) if device is not None else tensors[0].device
    res = parafac_epc_many([t.to(dev) for t in tensors], [int(r) for r in ranks], init="random", als_maxiter=50,
                           epc_maxiter=50)
    return [[f.to(device=dev, dtype=torch.float32) for f in us] for _, us in res]


def _problem(H, U, F, G, HT_out=None, X_out=None):
    I, R = H.shape
    if F.shape != (I, R) or U.shape != (I, R) or G.shape != (R, R):
        raise ValueError(f"admm_iteration: shape mismatch H{tuple(H.shape)} U{tuple(U.shape)} "
                         f"F{tuple(F.shape)} G{tuple(G.shape)}")
    return _lib.AdmmProblem(F.data_ptr(), G.data_ptr(), H.data_ptr(), 0, U.data_ptr(),
                            0 if HT_out is None else HT_out.data_ptr(), 0 if X_out is None else X_out.data_ptr(),
                            I, R)


def admm_iteration_batched(problems: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]],
                           max_iter: int, eps: float, bits: int, qscheme: str, num_attempts: int = 200,
                           check_spd: bool = True, debug_outputs: bool = False, return_info: bool = False,
                           solve: Optional[str] = None, check_fault: bool = True):
    """Run ``admm_iteration`` on every (H, U, F, G) of ``problems`` in shared launches.

    Returns the list of new H tensors (and the caller's U tensors are updated in
    place). With ``return_info`` also returns an int32 tensor [n, 5] of
    {iterations run, converged, spd_error, internal fault, re-runs of this call} (the
    last column is 1 when an internal fault was repaired; ``_lib.fault_repairs`` counts
    them process-wide); with ``debug_outputs`` a list
    of (H_T, X) of the last iteration per problem. ``solve``: ``"fp32"`` (the process
    default unless ``_lib.solve_mode`` changed it: fp32 MFMA, the reference's arithmetic)
    or ``"split"`` for this call. Calls ``torch.ops.admmq.admm_iteration_batched``
    (csrc/torch_ops.cpp), which calls ``admmq_admm_prepare_ex`` / ``admmq_admm_run_ex``;
    an internal fault of the fused finalize (its bounded wait timed out) is repaired
    inside the call by a re-run with the separate finalize launch (one host sync per call).
    ``check_fault=False`` skips that sync (calls on several streams can then overlap): the
    caller must read ``info[:, 3]`` itself and repeat the call with ``U`` restored where it
    is nonzero (``return_info`` is then required).
    """
    if not check_fault and not return_info:
        raise ValueError("check_fault=False needs return_info=True (the caller must check info[:, 3])")
    solve_code = -1 if solve is None else _lib.SOLVE_MODES[solve]
    if len(problems) == 0:
        return []
    for (H, U, F, G) in problems:
        _lib.require_device(H, U, F, G)
        if H.dim() != 2:
            raise ValueError("admm_iteration expects 2-D factors (I, R)")
    code = _scheme_code(qscheme)
    if not _lib.use_ops():
        return _admm_iteration_batched_cabi(problems, max_iter, eps, bits, code, num_attempts, check_spd,
                                            debug_outputs, return_info, solve_code, check_fault)
    Hs, Us, Fs, Gs = (list(x) for x in zip(*problems))
    outs, info, hts, xs = _lib.ops().admm_iteration_batched(Hs, Us, Fs, Gs, int(max_iter), float(eps), int(bits), code,
                                                            int(num_attempts), bool(check_spd), bool(debug_outputs),
                                                            solve_code, bool(check_fault))
    ret = [list(outs) if max_iter > 1 else [p[0] for p in problems]]   # max_iter <= 1: the input H objects
    if debug_outputs:
        ret.append(list(zip(hts, xs)))
    if return_info:
        ret.append(info)
    return ret[0] if len(ret) == 1 else tuple(ret)


def _admm_iteration_batched_cabi(problems, max_iter, eps, bits, code, num_attempts, check_spd, debug_outputs,
                                 return_info, solve_code=-1, check_fault=True):
    """The same call through the C-ABI with ctypes (diagnostic builds, cross-checks),
    including the op's internal-fault repair (restore U, re-run without the fused finalize)."""
    import ctypes
    lib = _lib.load()
    dev = problems[0][0].device
    Hs = [p[0].contiguous() for p in problems]
    Fs = [p[2].contiguous() for p in problems]
    Gs = [p[3].contiguous() for p in problems]
    Us_user = [p[1] for p in problems]
    Us = [u if u.is_contiguous() else u.contiguous() for u in Us_user]
    dbg = [(torch.empty_like(h), torch.empty_like(h)) for h in Hs] if debug_outputs else [(None, None)] * len(Hs)
    items = [_problem(H, U, F, G, *d) for H, U, F, G, d in zip(Hs, Us, Fs, Gs, dbg)]
    n = len(items)
    opt = _lib.default_options()
    if solve_code >= 0:
        opt.solve_mode = solve_code
    po = ctypes.byref(opt)
    arr = _lib.problems_array(items)
    nb = lib.admmq_admm_workspace_size_ex(arr, n, int(num_attempts), po)
    if nb == 0:
        _lib.check(-1, "admm workspace planning")
    ws = _lib.workspace(nb, dev)
    stream = _lib.stream_handle(dev)
    _lib.check(lib.admmq_admm_prepare_ex(arr, n, int(num_attempts), po, _lib.ptr(ws), nb, stream), "admm_prepare")
    info = torch.zeros(n * 4, dtype=torch.int32, device=dev)
    if check_spd or max_iter <= 1:
        # source/admm.py:54 raises before anything is modified: sync once per call
        _lib.check(lib.admmq_admm_run_ex(arr, n, 1, 0.0, 4, 0, int(num_attempts), po, _lib.ptr(ws), nb, _lib.ptr(info),
                                         stream), "admm_info")
        if int(info.view(n, 4)[:, 2].max().item()) != 0:
            raise torch.linalg.LinAlgError("linalg.cholesky: The factorization could not be completed because "
                                           "the input is not positive-definite.")
    def info5(reruns=0):
        out = torch.zeros((n, 5), dtype=torch.int32, device=dev)
        out[:, :4] = info.view(n, 4)
        out[:, 4] = reruns
        return out

    if max_iter <= 1:
        outs = [p[0] for p in problems]
        return (outs, info5()) if return_info else outs
    outs = [torch.empty_like(h) for h in Hs]
    for it, o in zip(items, outs):
        it.H_out = o.data_ptr()
    arr = _lib.problems_array(items)
    ubak = [u.clone() for u in Us] if check_fault else []

    def run():
        _lib.check(lib.admmq_admm_run_ex(arr, n, int(max_iter), float(eps), int(bits), code, int(num_attempts), po,
                                         _lib.ptr(ws), nb, _lib.ptr(info), stream), "admm_run")

    run()
    reruns = 0
    if check_fault and int(info.view(n, 4)[:, 3].max().item()) != 0:   # internal fault: repeat without the fused finalize
        for u, b in zip(Us, ubak):
            u.copy_(b)
        opt.fused_finalize = 0
        _lib.check(lib.admmq_admm_prepare_ex(arr, n, int(num_attempts), po, _lib.ptr(ws), nb, stream), "admm_prepare")
        run()
        if int(info.view(n, 4)[:, 3].max().item()) != 0:
            raise RuntimeError("admmq: internal fault in the separate-finalize re-run")
        reruns = 1
        _lib.note_repair()
    for u_user, u in zip(Us_user, Us):
        if u is not u_user:
            u_user.copy_(u)
    ret = [outs]
    if debug_outputs:
        ret.append(dbg)
    if return_info:
        ret.append(info5(reruns))
    return ret[0] if len(ret) == 1 else tuple(ret)


def admm_iteration(H: torch.Tensor, U: torch.Tensor, F: torch.Tensor, G: torch.Tensor, max_iter: int, eps: float,
                   bits: int, qscheme: str, num_attempts: int = 200, solve: Optional[str] = None):
    """source/admm.py:51-67 -> (H_new, U)."""
    out = admm_iteration_batched([(H, U, F, G)], max_iter, eps, bits, qscheme, num_attempts=num_attempts, solve=solve)
    return out[0], U
