"""Panel products of the device rank projection (``scripts/factorize_lowrank.py:80-82``).

``xtq(X, Q) = X^T Q``, ``xy(X, Y) = X Y`` and ``outer(A, B) = A B^T`` over the C-ABI
(``admmq_panel_*``, ``csrc/panel_kernels.hip``): X is the low-rank loop's float32 iterate,
read once per product and widened to float64 in registers (v_mfma_f64_16x16x4_f64, fp64
accumulation in an order fixed by the shapes); the panels are float64. There is no
fallback: the HIP library must be loaded.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional, Tuple

import torch

from . import _lib

# Workspaces keyed by (device, stream): the panel kernels' cross-workgroup partials and
# arrival counters (which only count up; the workgroup that finishes a tile is the one whose
# add completes a multiple of the group size) require every call on one workspace to be
# stream-ordered (include/admmq.h). One workspace per stream keeps calls on different
# streams from racing on the same slots and counters. A workspace is allocated on its own
# stream, so when it is grown the caching allocator reuses the old block only for later work
# of that same stream - never while another stream's kernel may still read it.
_WS: "OrderedDict[Tuple[torch.device, int], torch.Tensor]" = OrderedDict()
_GWS: "OrderedDict[Tuple[torch.device, int], torch.Tensor]" = OrderedDict()


def _key(dev: torch.device) -> Tuple[torch.device, int]:
    return (dev, int(torch.cuda.current_stream(dev).cuda_stream))


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    """The partials / arrival counters of the panel kernels, per (device, current stream),
    grown on demand and zeroed when (re)allocated (the counters must start at a multiple of
    the group size)."""
    return _cached(_WS, dev, nbytes, zero=True)


def _check_x(X: torch.Tensor) -> torch.Tensor:
    if not isinstance(X, torch.Tensor) or X.device.type != "cuda":
        raise RuntimeError("admmq.panel: X must be a tensor on a ROCm GPU (no CPU implementation)")
    if X.dim() != 2 or X.dtype != torch.float32:
        raise ValueError("admmq.panel: X must be a 2-D float32 device tensor")
    return X if X.stride(1) == 1 else X.contiguous()


def _check_panel(P: torch.Tensor, rows: int, X: torch.Tensor, name: str) -> torch.Tensor:
    if P.dim() != 2 or P.shape[0] != rows or P.dtype != torch.float64 or P.device != X.device:
        raise ValueError(f"admmq.panel: {name} must be a float64 tensor with {rows} rows on X's device")
    return P.contiguous()


def xtq(X: torch.Tensor, Q: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``X^T Q`` (n x k float64) for X m x n float32, Q m x k float64."""
    X = _check_x(X)
    m, n = X.shape
    Q = _check_panel(Q, m, X, "Q")
    k = Q.shape[1]
    Y = out if out is not None else torch.empty(n, k, dtype=torch.float64, device=X.device)
    lib = _lib.load()
    nb = lib.admmq_panel_workspace_size(m, n, k)
    ws = _workspace(X.device, nb)
    _lib.check(lib.admmq_panel_xtq(_lib.ptr(X), m, n, X.stride(0), _lib.ptr(Q), k, _lib.ptr(Y), _lib.ptr(ws),
                                   ws.numel(), _lib.stream_handle(X.device)), "panel_xtq")
    return Y


def xy(X: torch.Tensor, Y: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``X Y`` (m x k float64) for X m x n float32, Y n x k float64."""
    X = _check_x(X)
    m, n = X.shape
    Y = _check_panel(Y, n, X, "Y")
    k = Y.shape[1]
    Z = out if out is not None else torch.empty(m, k, dtype=torch.float64, device=X.device)
    lib = _lib.load()
    nb = lib.admmq_panel_workspace_size(m, n, k)
    ws = _workspace(X.device, nb)
    _lib.check(lib.admmq_panel_xy(_lib.ptr(X), m, n, X.stride(0), _lib.ptr(Y), k, _lib.ptr(Z), _lib.ptr(ws),
                                  ws.numel(), _lib.stream_handle(X.device)), "panel_xy")
    return Z


def outer(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``A B^T`` rounded once to float32 (m x n) for A m x r, B n x r float64, r <= 32."""
    if not isinstance(A, torch.Tensor) or not isinstance(B, torch.Tensor) or A.device.type != "cuda" or B.device != A.device:
        raise RuntimeError("admmq.panel.outer: A and B must be tensors on one ROCm GPU")
    if A.dim() != 2 or B.dim() != 2 or A.shape[1] != B.shape[1] or A.dtype != torch.float64 or B.dtype != torch.float64:
        raise ValueError("admmq.panel.outer: A (m x r) and B (n x r) float64 with one r")
    A, B = A.contiguous(), B.contiguous()
    m, r = A.shape
    n = B.shape[0]
    O = out if out is not None else torch.empty(m, n, dtype=torch.float32, device=A.device)
    _lib.check(_lib.load().admmq_panel_outer(_lib.ptr(A), _lib.ptr(B), m, n, r, _lib.ptr(O), O.stride(0),
                                             _lib.stream_handle(A.device)), "panel_outer")
    return O


def gram(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``A^T B`` (p x q float64) for tall A (m x p) and B (m x q) float64 on one device."""
    if not isinstance(A, torch.Tensor) or not isinstance(B, torch.Tensor) or A.device.type != "cuda" or B.device != A.device:
        raise RuntimeError("admmq.panel.gram: A and B must be tensors on one ROCm GPU")
    if A.dim() != 2 or B.dim() != 2 or A.shape[0] != B.shape[0] or A.dtype != torch.float64 or B.dtype != torch.float64:
        raise ValueError("admmq.panel.gram: A (m x p) and B (m x q) float64 with one m")
    A = A if A.stride(1) == 1 else A.contiguous()
    B = B if B.stride(1) == 1 else B.contiguous()
    m, p = A.shape
    q = B.shape[1]
    C = out if out is not None else torch.empty(p, q, dtype=torch.float64, device=A.device)
    lib = _lib.load()
    nb = lib.admmq_gram64_workspace_size(m, p, q)
    ws = _cached(_GWS, A.device, nb, zero=False)
    _lib.check(lib.admmq_gram64(_lib.ptr(A), A.stride(0), _lib.ptr(B), B.stride(0), m, p, q, _lib.ptr(C), _lib.ptr(ws),
                                ws.numel(), _lib.stream_handle(A.device)), "gram64")
    return C


def epc_mu(c: torch.Tensor, s: torch.Tensor, normY2: float, delta2: float) -> torch.Tensor:
    """The EPC multiplier (``admmq.parafac_epc._solve_mu``) on the device: a 0-dim float64
    tensor, with no host synchronisation."""
    if c.dtype != torch.float64 or s.dtype != torch.float64 or c.shape != s.shape or c.dim() != 1:
        raise ValueError("admmq.panel.epc_mu: c and s must be float64 vectors of one length")
    c, s = c.contiguous(), s.contiguous()
    mu = torch.empty((), dtype=torch.float64, device=c.device)
    _lib.check(_lib.load().admmq_epc_mu(_lib.ptr(c), _lib.ptr(s), c.numel(), float(normY2), float(delta2), _lib.ptr(mu),
                                        _lib.stream_handle(c.device)), "epc_mu")
    return mu


def colnorm64(A: torch.Tensor, B: Optional[torch.Tensor] = None):
    """cp_anc's normalisation of the other factors in one launch: ``A / max(||A[:, r]||, 1e-300)``
    per column (and B likewise); new tensors, the inputs untouched (float64, contiguous, on
    the device, the same number of columns)."""
    for t in (A, B):
        if t is not None and (t.dtype != torch.float64 or t.dim() != 2 or t.device.type != "cuda"):
            raise ValueError("admmq.panel.colnorm64: float64 2-D device tensors")
    if B is not None and B.shape[1] != A.shape[1]:
        raise ValueError("admmq.panel.colnorm64: A and B need the same number of columns")
    A = A.contiguous()
    B = B.contiguous() if B is not None else None
    oA = torch.empty_like(A)
    oB = torch.empty_like(B) if B is not None else None
    _lib.check(_lib.load().admmq_cp_colnorm64(_lib.ptr(A), A.shape[0], _lib.ptr(B) if B is not None else None,
                                              B.shape[0] if B is not None else 0, A.shape[1], _lib.ptr(oA),
                                              _lib.ptr(oB) if oB is not None else None,
                                              _lib.stream_handle(A.device)), "cp_colnorm64")
    return oA, oB


SPD_SMALL_MAX = 136   # n of the one-workgroup fp64 solves (csrc/epc_kernels.hip: the matrix in LDS)
EPC_FIRST_ROUNDS = 3   # blocked EPC step: evaluation rounds queued before the first read of its done flag
EPC_NEXT_ROUNDS = 2    # ... and between later reads

_SWS: "OrderedDict[Tuple[torch.device, int], torch.Tensor]" = OrderedDict()   # blocked-solve workspaces
_CACHE_MAX = 64   # workspaces kept per cache (least recently used dropped; see _cached)


def _cached(cache, dev: torch.device, nbytes: int, zero: bool) -> torch.Tensor:
    """The workspace of the current stream (grown on demand). At most _CACHE_MAX streams keep one:
    the least recently used is released to the caching allocator, which reuses a block only for
    later work of the stream it was allocated on, so a kernel still queued there is safe."""
    k = _key(dev)
    ws = cache.get(k)
    if ws is None or ws.numel() < nbytes:
        ws = (torch.zeros if zero else torch.empty)(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
        cache[k] = ws
    cache.move_to_end(k)
    while len(cache) > _CACHE_MAX:
        cache.popitem(last=False)
    return ws


def _check_solve(G: torch.Tensor, F: torch.Tensor, what: str):
    n = G.shape[0]
    if G.dtype != torch.float64 or F.dtype != torch.float64 or G.shape != (n, n) or F.dim() != 2 or F.shape[1] != n:
        raise ValueError(f"admmq.panel.{what}: G (n x n) and F (m x n) must be float64")
    if G.device.type != "cuda" or F.device != G.device:
        raise RuntimeError(f"admmq.panel.{what}: G and F must be on one ROCm GPU (no CPU implementation)")
    return G.contiguous(), F.contiguous()


def _info_ptr(info: Optional[torch.Tensor]):
    if info is None:
        return None
    if info.dtype != torch.int32 or info.numel() != 1 or info.device.type != "cuda":
        raise ValueError("admmq.panel: info must be a one-element int32 device tensor")
    return _lib.ptr(info)


def spd_solve64(G: torch.Tensor, F: torch.Tensor, info: Optional[torch.Tensor] = None,
                rel_shift: float = 0.0) -> torch.Tensor:
    """``F (G + rel_shift (tr G / n) I)^-1`` (m x n float64) for SPD ``G`` on the device: the CP-ALS
    update ``torch.linalg.solve(G, F.T).T`` of tensorly ``parafac``, with no host synchronisation.
    n <= SPD_SMALL_MAX: one workgroup, an unpivoted blocked Gauss-Jordan inverse in LDS; larger n:
    the blocked fp64 Cholesky L L^T, L^-1 and X = (F L^-T) L^-1 on fp64 MFMA
    (``csrc/solve64.hip``). A G that is not numerically positive definite sets ``info`` (a
    one-element int32 device tensor) to 1 and leaves X undefined; without ``info`` it goes
    unnoticed, so the drivers always pass one (``admmq.parafac_epc`` retries such an update
    with a small relative shift)."""
    G, F = _check_solve(G, F, "spd_solve64")
    m, n = F.shape
    X = torch.empty(F.shape, dtype=torch.float64, device=F.device)
    if m == 0:
        return X
    lib = _lib.load()
    ws = None
    nb = 0
    if n > SPD_SMALL_MAX:
        nb = lib.admmq_solve64_workspace_size(m, n)
        ws = _cached(_SWS, F.device, nb, zero=False)
    _lib.check(lib.admmq_spd_solve64_ws(_lib.ptr(G), _lib.ptr(F), m, n, float(rel_shift), _lib.ptr(X), _info_ptr(info),
                                        _lib.ptr(ws) if ws is not None else None, ws.numel() if ws is not None else 0,
                                        _lib.stream_handle(F.device)), "spd_solve64")
    return X


def epc_step64(G: torch.Tensor, F: torch.Tensor, normY2: float, delta2: float, mu: torch.Tensor,
               info: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One EPC mode update of musco ``cp_anc`` on the device: ``F (G + mu I)^-1`` with ``mu >= 0``
    the root of the error equation. ``mu`` is a 0-dim float64 device tensor: the warm start in,
    the root out (updated in place). n <= SPD_SMALL_MAX: one launch (``csrc/epc_kernels.hip``: G
    tridiagonalised once, then safeguarded Newton steps on tridiagonal L D L^T recurrences; no
    host synchronisation); larger n: the blocked step (``epc_step64_gen``), driven to completion
    here. ``info`` (one-element int32 device tensor): 0, or 1 when no G + mu I on the search
    bracket was positive definite or the search did not converge."""
    if G.shape[0] > SPD_SMALL_MAX:
        gen = epc_step64_gen(G, F, normY2, delta2, mu, info)
        try:
            ev = next(gen)
            while True:
                ev.synchronize()
                ev = gen.send(None)
        except StopIteration as stop:
            return stop.value
    G, F = _check_solve(G, F, "epc_step64")
    n = G.shape[0]
    if mu.dtype != torch.float64 or mu.numel() != 1 or mu.device != F.device:
        raise ValueError("admmq.panel.epc_step64: mu must be a float64 scalar tensor on F's device")
    X = torch.empty(F.shape, dtype=torch.float64, device=F.device)
    work = torch.empty(F.shape, dtype=torch.float64, device=F.device)
    _lib.check(_lib.load().admmq_epc_step64(_lib.ptr(G), _lib.ptr(F), F.shape[0], n, float(normY2), float(delta2),
                                            _lib.ptr(mu), _lib.ptr(X), _lib.ptr(work), _info_ptr(info),
                                            _lib.stream_handle(F.device)),
               "epc_step64")
    return X


def epc_step64_gen(G: torch.Tensor, F: torch.Tensor, normY2: float, delta2: float, mu: torch.Tensor,
                   info: Optional[torch.Tensor] = None):
    """The blocked EPC step for any n (``csrc/solve64.hip``) as a generator: it queues evaluation
    rounds (each a Cholesky of G + mu I at the search's next mu and the Newton update, all on the
    device) and yields a ``torch.cuda.Event`` whenever it needs the done flag on the host
    (``EPC_FIRST_ROUNDS`` rounds, then ``EPC_NEXT_ROUNDS`` per read); resume it once the event has
    completed. Returns X = F (G + mu I)^-1; ``mu`` updated in place, ``info`` as ``epc_step64``.
    The step's search state lives in the current stream's cached workspace, so one stream runs
    one blocked step (or blocked solve) at a time: finish this generator before the next such
    call on its stream. ``admmq.parafac_epc`` drives several of these at once, one layer per
    stream."""
    G, F = _check_solve(G, F, "epc_step64")
    m, n = F.shape
    if mu.dtype != torch.float64 or mu.numel() != 1 or mu.device != F.device:
        raise ValueError("admmq.panel.epc_step64: mu must be a float64 scalar tensor on F's device")
    lib = _lib.load()
    dev = F.device
    X = torch.empty(F.shape, dtype=torch.float64, device=dev)
    nb = lib.admmq_solve64_workspace_size(m, n)
    ws = _cached(_SWS, dev, nb, zero=False)
    done = torch.zeros(1, dtype=torch.int32, device=dev)
    st = _lib.stream_handle(dev)
    _lib.check(lib.admmq_epc_begin64(_lib.ptr(G), _lib.ptr(F), m, n, float(normY2), float(delta2), _lib.ptr(mu),
                                     _lib.ptr(X), _lib.ptr(ws), ws.numel(), st), "epc_begin64")
    rounds, total = EPC_FIRST_ROUNDS, 0
    while total < 96:   # the device search's evaluation budget (kS64MaxEvals, csrc/solve64.hip)
        _lib.check(lib.admmq_epc_rounds64(_lib.ptr(G), _lib.ptr(F), m, n, _lib.ptr(X), rounds, _lib.ptr(done),
                                          _lib.ptr(ws), ws.numel(), st), "epc_rounds64")
        total += rounds
        host = done.to("cpu", non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        yield ev
        if int(host[0]):
            break
        rounds = EPC_NEXT_ROUNDS
    _lib.check(lib.admmq_epc_end64(m, n, _lib.ptr(mu), _info_ptr(info), _lib.ptr(ws), ws.numel(), st), "epc_end64")
    return X
