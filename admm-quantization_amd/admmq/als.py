"""ALS-sweep contractions on the MI355X (C-ABI ``admmq_cp_gram_mttkrp`` / ``admmq_cp_rel_error``).

* ``gram_mttkrp(W, factors, mode)`` -> ``(G, F)``: the per-mode setup of
  ``scripts/factorize.py:215-237`` (3-way: ``G = B.T @ B * (C.T @ C)``,
  ``F = torch.einsum('abc,cr,br->ar', W, C, B)`` and the B / C analogues) and
  ``:276-287`` (2-way: ``G = B.T @ B``, ``F = W @ B``; ``G = A.T @ A``, ``F = W.T @ A``).
* ``rel_error(W, factors)``: ``squared_relative_diff(W, torch.einsum('ir,jr,kr->ijk', A, B, C))``
  of ``scripts/factorize.py:246-253`` / ``source/admm.py:14-15`` without building the
  reconstruction.

The ``*_batched`` forms take many layers in one launch sequence (the ALS driver
solves mode m of every layer together). HIP only: CPU tensors raise.

* ``gram_mttkrp_f64(Y, factors, mode)`` -> ``(F, G)``: the same per-mode contractions in
  fp64 (C-ABI ``admmq_cp64_gram_mttkrp``, f64 MFMA) for the CP-ALS / EPC initialiser
  (``admmq.parafac_epc``; tensorly ``parafac`` / musco ``cp_anc`` in the reference,
  ``source/parafac_epc.py:42-74``).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib


def _validate(W: torch.Tensor, factors: Sequence[torch.Tensor]):
    if W.dim() not in (2, 3):
        raise ValueError(f"admmq: CP layer tensor must be 2-D or 3-D, got {W.dim()}-D")
    if len(factors) != W.dim():
        raise ValueError(f"admmq: {W.dim()}-way tensor needs {W.dim()} factors, got {len(factors)}")
    R = factors[0].shape[1]
    for d, f in enumerate(factors):
        if f.dim() != 2 or f.shape != (W.shape[d], R):
            raise ValueError(f"admmq: factor {d} has shape {tuple(f.shape)}, expected {(W.shape[d], R)}")
    _lib.require_device(W, *factors)
    return R


def _layer(W: torch.Tensor, factors: Sequence[torch.Tensor], G: Optional[torch.Tensor] = None,
           F: Optional[torch.Tensor] = None) -> _lib.CpLayer:
    R = _validate(W, factors)
    L = _lib.CpLayer()
    L.W = W.data_ptr()
    for d in range(3):
        L.factors[d] = factors[d].data_ptr() if d < len(factors) else None
    L.G = G.data_ptr() if G is not None else None
    L.F = F.data_ptr() if F is not None else None
    for d in range(3):
        L.dims[d] = W.shape[d] if d < W.dim() else 0
    L.ndim = W.dim()
    L.R = R
    return L


def gram_mttkrp_batched(layers: Sequence[Tuple[torch.Tensor, Sequence[torch.Tensor]]], mode: int
                        ) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """``[(G, F)]`` for mode ``mode`` of every ``(W, factors)`` (factors[mode] is not read)."""
    if not layers:
        return []
    if _lib.use_ops():   # torch.ops.admmq.cp_gram_mttkrp (csrc/torch_ops.cpp) -> admmq_cp_gram_mttkrp
        for W, fs in layers:
            _validate(W, fs)
            if not 0 <= mode < W.dim():
                raise ValueError(f"admmq: mode {mode} out of range for a {W.dim()}-way tensor")
        G, F = _lib.ops().cp_gram_mttkrp([W for W, _ in layers], [f for _, fs in layers for f in fs], int(mode))
        return list(zip(G, F))
    lib = _lib.load()
    keep, outs, descs = [], [], []
    for W, fs in layers:
        W = W.contiguous()
        fs = [f.contiguous() for f in fs]
        if not 0 <= mode < W.dim():
            raise ValueError(f"admmq: mode {mode} out of range for a {W.dim()}-way tensor")
        R = fs[0].shape[1]
        G = torch.empty(R, R, dtype=torch.float32, device=W.device)
        F = torch.empty(W.shape[mode], R, dtype=torch.float32, device=W.device)
        descs.append(_layer(W, fs, G, F))
        keep.append((W, fs))
        outs.append((G, F))
    arr = (_lib.CpLayer * len(descs))(*descs)
    dev = layers[0][0].device
    nbytes = lib.admmq_cp_workspace_size(arr, len(descs), mode)
    if nbytes == 0:
        _lib.check(-1, "cp_workspace_size")
    ws = _lib.workspace(nbytes, dev)
    _lib.check(lib.admmq_cp_gram_mttkrp(arr, len(descs), mode, _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev)),
               "cp_gram_mttkrp")
    del keep
    return outs


def gram_mttkrp(W: torch.Tensor, factors: Sequence[torch.Tensor], mode: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """G (Gram∘Gram) and F (MTTKRP) of one layer's mode ``mode``."""
    return gram_mttkrp_batched([(W, factors)], mode)[0]


def rel_error_batched(layers: Sequence[Tuple[torch.Tensor, Sequence[torch.Tensor]]],
                      as_tensor: bool = False):
    """``||W - [[factors]]||_F / ||W||_F`` per layer. One host sync for the whole batch
    (the reference syncs once per error through ``.item()``); ``as_tensor=True`` keeps the
    fp64 results on the device and does not sync."""
    if not layers:
        return torch.zeros(0, dtype=torch.float64) if as_tensor else []
    if _lib.use_ops():   # torch.ops.admmq.cp_rel_error (csrc/torch_ops.cpp) -> admmq_cp_rel_error
        for W, fs in layers:
            _validate(W, fs)
        out = _lib.ops().cp_rel_error([W for W, _ in layers], [f for _, fs in layers for f in fs])
        return out if as_tensor else [float(v) for v in out.cpu()]
    lib = _lib.load()
    keep, descs = [], []
    for W, fs in layers:
        W = W.contiguous()
        fs = [f.contiguous() for f in fs]
        descs.append(_layer(W, fs))
        keep.append((W, fs))
    arr = (_lib.CpLayer * len(descs))(*descs)
    dev = layers[0][0].device
    out = torch.empty(len(descs), dtype=torch.float64, device=dev)
    nbytes = lib.admmq_cp_workspace_size(arr, len(descs), 0)
    if nbytes == 0:
        _lib.check(-1, "cp_workspace_size")
    ws = _lib.workspace(nbytes, dev)
    _lib.check(lib.admmq_cp_rel_error(arr, len(descs), ctypes.c_void_p(out.data_ptr()), _lib.ptr(ws), ws.numel(),
                                      _lib.stream_handle(dev)), "cp_rel_error")
    del keep
    if as_tensor:
        return out
    return [float(v) for v in out.cpu()]


def rel_error(W: torch.Tensor, factors: Sequence[torch.Tensor]) -> float:
    return rel_error_batched([(W, factors)])[0]


def gram_mttkrp_f64(Y: torch.Tensor, factors: Sequence[torch.Tensor], mode: int
                    ) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp64 ``(F, G)`` of mode ``mode``: F = Y_(mode) . KR(other factors) (torch ``unfold``
    / Khatri-Rao order), G = Hadamard product of the other factors' Grams. factors[mode]
    is not read. Float64 tensors on the GPU only."""
    if Y.dim() not in (2, 3):
        raise ValueError(f"admmq: CP tensor must be 2-D or 3-D, got {Y.dim()}-D")
    if len(factors) != Y.dim():
        raise ValueError(f"admmq: {Y.dim()}-way tensor needs {Y.dim()} factors, got {len(factors)}")
    R = factors[0].shape[1]
    for d, f in enumerate(factors):
        if f.dim() != 2 or f.shape != (Y.shape[d], R):
            raise ValueError(f"admmq: factor {d} has shape {tuple(f.shape)}, expected {(Y.shape[d], R)}")
    for t in (Y, *factors):
        if t.device.type != "cuda" or t.dtype != torch.float64:
            raise RuntimeError("admmq: the fp64 CP contractions need float64 tensors on a ROCm GPU (no CPU path)")
    Y = Y.contiguous()
    fs = [f.contiguous() for f in factors]
    F = torch.empty(Y.shape[mode], R, dtype=torch.float64, device=Y.device)
    G = torch.empty(R, R, dtype=torch.float64, device=Y.device)
    L = _lib.CpLayer()   # admmq_cp_layer_f64 has admmq_cp_layer's layout
    L.W = Y.data_ptr()
    for d in range(3):
        L.factors[d] = fs[d].data_ptr() if d < len(fs) else None
        L.dims[d] = Y.shape[d] if d < Y.dim() else 0
    L.G, L.F, L.ndim, L.R = G.data_ptr(), F.data_ptr(), Y.dim(), R
    lib = _lib.load()
    arr = (_lib.CpLayer * 1)(L)
    nbytes = lib.admmq_cp64_workspace_size(arr, 1, mode)
    if nbytes == 0:
        _lib.check(1, "cp64_workspace_size")
    ws = _lib.workspace(nbytes, Y.device)
    _lib.check(lib.admmq_cp64_gram_mttkrp(arr, 1, mode, _lib.ptr(ws), ws.numel(), _lib.stream_handle(Y.device)),
               "cp64_gram_mttkrp")
    return F, G
