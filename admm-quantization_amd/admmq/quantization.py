"""Drop-in quantizers (``source/quantization.py:12-144``) on the MI355X.

``quantize_tensor(tensor, bits, qscheme, dim=None, **kwargs)`` keeps the
reference's names, argument meaning and error behaviour:

* ``tensor_mseminmax_symmetric`` -> 200-candidate MSE-minmax search
  (``quantize_tensor_mse``, :118-144; ``num_attempts`` via kwargs);
* ``tensor_minmax`` -> ``min_max_quantize`` (:48-66);
* ``tensor_symmetric`` / ``tensor_affine`` -> :91-106 (``tmin``/``tmax`` kwargs);
* ``channel_symmetric`` / ``channel_affine`` with an explicit ``dim`` -> per-channel
  statistics of ``unfold(tensor, dim)`` broadcast against the tensor's last dimension,
  exactly as the reference's torch code does (:29-33, 91-106; an incompatible size raises
  the same ``RuntimeError``); ``dim=None`` raises ``TypeError`` (the reference fails in
  ``unfold(tensor, None)``); ``tensor_log`` and unknown names raise
  ``NotImplementedError``.

All arithmetic runs in the HIP library (``libadmmq.so``); the MSE reduction
follows the canonical fixed-point rule documented in ``DESIGN.md`` §3, which is
order-independent and therefore bit-identical between runs, grids and the CPU
oracle.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import _lib

__all__ = ["quantize_tensor", "quantize_channel", "quantize_tensor_mse", "min_max_quantize", "quantize_batched", "get_tensor_stats",
           "mse_sse_table"]


def _scheme_code(qscheme: str, dim=None) -> int:
    if qscheme in _lib.CHANNEL_SCHEMES:
        if dim is None:
            raise TypeError("Can't collect per-channel statistics with dim=None "
                            "(reference: unfold(tensor, mode=None))")
        return _lib.CHANNEL_SCHEMES[qscheme]
    if qscheme not in _lib.SCHEMES:
        raise NotImplementedError(qscheme)
    return _lib.SCHEMES[qscheme]


def _rows_cols(t: torch.Tensor):
    if t.dim() == 0:
        return 1, 1
    cols = t.shape[-1]
    return t.numel() // cols, cols


def quantize_batched(tensors: Sequence[torch.Tensor], bits: int, qscheme: str, num_attempts: int = 200,
                     tmin: Optional[float] = None, tmax: Optional[float] = None) -> List[torch.Tensor]:
    """Quantize several tensors with one launch sequence (one job per tensor)."""
    code = _scheme_code(qscheme)
    lib = _lib.load()
    if bits < 1:
        raise AssertionError(bits)
    xs = []
    for t in tensors:
        _lib.require_device(t)
        if t.numel() == 0:
            raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0.")
        xs.append(t.contiguous())
    if _lib.use_ops():   # torch.ops.admmq.quantize_batched (csrc/torch_ops.cpp) -> admmq_quantize_batched
        has_kw = code == 3 and tmin is not None and tmax is not None
        return list(_lib.ops().quantize_batched(xs, int(bits), code, int(num_attempts),
                                                float(tmin) if has_kw else None, float(tmax) if has_kw else None))
    dev = xs[0].device
    outs = [torch.empty_like(x) for x in xs]
    items = []
    has_kw = code == 3 and tmin is not None and tmax is not None
    for x, y in zip(xs, outs):
        r, c = _rows_cols(x)
        items.append(_lib.QTensor(x.data_ptr(), y.data_ptr(), r, c, float(tmin) if has_kw else 0.0,
                                  float(tmax) if has_kw else 0.0, 1 if has_kw else 0, 0))
    arr = _lib.qtensor_array(items)
    nb = lib.admmq_quantize_workspace_size(arr, len(items), int(num_attempts))
    if nb == 0:
        _lib.check(-1, "quantize workspace planning")
    ws = _lib.workspace(nb, dev)
    rc = lib.admmq_quantize_batched(arr, len(items), int(bits), code, int(num_attempts), _lib.ptr(ws), nb,
                                    _lib.stream_handle(dev))
    _lib.check(rc, "quantize_batched")
    return outs


def quantize_channel(tensor: torch.Tensor, bits: int, qscheme: str, dim: int) -> torch.Tensor:
    """``channel_symmetric`` / ``channel_affine`` with an explicit ``dim``
    (``source/quantization.py:29-33, 91-106``) on the device (``admmq_quantize_channel``)."""
    code = _scheme_code(qscheme, dim)
    _lib.require_device(tensor)
    if bits < 1:
        raise AssertionError(bits)
    if tensor.dim() == 0:
        raise IndexError(f"Dimension out of range (expected to be in range of [-1, 0], but got {dim})")
    x = tensor.contiguous()
    if _lib.use_ops():
        return _lib.ops().quantize_channel(x, int(bits), code, int(dim))
    import ctypes
    lib = _lib.load()
    nd = x.dim()
    d = dim + nd if dim < 0 else dim
    if not 0 <= d < nd:
        raise IndexError(f"Dimension out of range (expected to be in range of [{-nd}, {nd - 1}], but got {dim})")
    C, L = x.shape[d], x.shape[-1]
    if L != C and L != 1 and C != 1:
        raise RuntimeError(f"The size of tensor a ({L}) must match the size of tensor b ({C}) at non-singleton "
                           f"dimension {nd - 1}")
    shape = (ctypes.c_int64 * nd)(*x.shape)
    y = torch.empty(tuple(x.shape[:-1]) + (max(L, C),), dtype=x.dtype, device=x.device)
    nb = lib.admmq_quantize_channel_workspace_size(shape, nd, d)
    ws = _lib.workspace(nb, x.device)
    _lib.check(lib.admmq_quantize_channel(_lib.ptr(x), _lib.ptr(y), shape, nd, d, int(bits), code, _lib.ptr(ws), nb,
                                          _lib.stream_handle(x.device)), "quantize_channel")
    return y


def quantize_tensor(tensor: torch.Tensor, bits: int, qscheme: str, dim=None, **kwargs) -> torch.Tensor:
    """source/quantization.py:69-115."""
    code = _scheme_code(qscheme, dim)
    if code in (4, 5):
        if code == 5 and kwargs.get("tmin") is not None and kwargs.get("tmax") is not None:
            # explicit range: the statistics are not collected, so the channel scheme is the
            # tensor scheme with that range (source/quantization.py:98-101)
            return quantize_tensor(tensor, bits, "tensor_affine", tmin=kwargs["tmin"], tmax=kwargs["tmax"])
        return quantize_channel(tensor, bits, qscheme, dim)
    num_attempts = int(kwargs.get("num_attempts", 200)) if code == 0 else 200
    tmin = kwargs.get("tmin") if code == 3 else None
    tmax = kwargs.get("tmax") if code == 3 else None
    if tmin is not None and tmax is not None:
        tmin, tmax = float(tmin), float(tmax)
    else:
        tmin = tmax = None
    return quantize_batched([tensor], bits, qscheme, num_attempts=num_attempts, tmin=tmin, tmax=tmax)[0]


def quantize_tensor_mse(x: torch.Tensor, bits: int, num_attempts: int = 200) -> torch.Tensor:
    """source/quantization.py:118-144."""
    return quantize_batched([x], bits, "tensor_mseminmax_symmetric", num_attempts=num_attempts)[0]


def min_max_quantize(input: torch.Tensor, bits: int, min_val=None, max_val=None) -> torch.Tensor:
    """source/quantization.py:48-66 (explicit min_val/max_val are not on the hot path)."""
    assert bits >= 1, bits
    if min_val is not None or max_val is not None:
        raise NotImplementedError("min_max_quantize with explicit range is outside the ADMM hot path")
    return quantize_batched([input], bits, "tensor_minmax")[0]


def get_tensor_stats(tensor: torch.Tensor, qscheme: str, mode=0):
    """source/quantization.py:12-45 (tensor schemes: (max, min) of all elements)."""
    if qscheme in ("channel_affine", "channel_symmetric"):
        if mode is None:
            raise TypeError("unfold(tensor, mode=None)")
        from .utils import unfold
        u = unfold(tensor, mode)
        return u.max(dim=-1)[0], u.min(dim=-1)[0]
    if qscheme in ("tensor_affine", "tensor_symmetric", "tensor_log"):
        return tensor.max(), tensor.min()
    raise TypeError("Can't collect statistics. Unknown quantization scheme: {}".format(qscheme))


def mse_sse_table(x: torch.Tensor, bits: int, num_attempts: int = 200) -> torch.Tensor:
    """Canonical per-candidate SSE (uint64 stored in int64) computed on the GPU (parity tests)."""
    _lib.require_device(x)
    lib = _lib.load()
    x = x.contiguous()
    r, c = _rows_cols(x)
    item = _lib.QTensor(x.data_ptr(), 0, r, c, 0.0, 0.0, 0, 0)
    arr = _lib.qtensor_array([item])
    nb = lib.admmq_quantize_workspace_size(arr, 1, int(num_attempts))
    ws = _lib.workspace(nb, x.device)
    out = torch.empty(int(num_attempts), dtype=torch.int64, device=x.device)
    rc = lib.admmq_mse_sse_table(_lib.ptr(x), r, c, int(bits), int(num_attempts), _lib.ptr(out), _lib.ptr(ws), nb,
                                 _lib.stream_handle(x.device))
    _lib.check(rc, "mse_sse_table")
    return out
