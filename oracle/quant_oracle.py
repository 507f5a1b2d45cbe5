"""ORACLE — test infrastructure only. CPU restatement of the reference quantizers.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker. The product path
(``admm-quantization_amd/admmq``) never imports it and fails loudly when the HIP
library is missing.

Pinned against the reference's own outputs: ``tests/golden/f1_quant.*`` and
``tests/golden/f5_linspace.npz`` were produced by importing
``/root/reference/source/quantization.py`` (see ``tests/golden/gen_golden.py``);
``tests/test_oracle_golden.py`` checks this module bit-for-bit against them.

Arithmetic is numpy float32 with IEEE division and round-half-even, i.e. the
same per-element operations torch-CPU performs in the reference.

The one place where the reference's result is not a pure function of the
per-element float32 operations is the MSE reduction (``.mean()`` over float32,
``source/quantization.py:138``), whose rounding depends on torch's CPU summation
order. The restatement replaces it by a *canonical, order-independent* rule that
the HIP kernel implements identically (so GPU == oracle bit-for-bit):

  * the tensor is viewed as (rows, last-dim) and each row is split into quads of 4
    consecutive elements (the last quad zero-padded);
  * per quad, g = fl32(fl32(d0²+d1²) + fl32(d2²+d3²)) with d = fl32(x − fl32(q·s));
  * g is converted to the fixed-point integer floor(g · 2^K) (exact in float64),
    K = 56 − ceil_log2(#quads) − 2·E where mx = m·2^E, m∈[0.5,1) (frexp);
  * SSE(candidate) = Σ of those integers in uint64 (associative => any order);
  * argmin takes the first index on ties (torch.argmin semantics).

This equals the exact float32-term SSE to ~2^-30 relative, far below the
float32 noise of the reference's own mean, and agrees with the reference on every
committed KAT (see the test for the count).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _f32(x):
    return np.float32(x)


def candidate_grid(mx: np.float32, n: int) -> np.ndarray:
    """torch.linspace(0.2*mx.item(), 1.2*mx.item(), n) as torch-CPU computes it
    (``source/quantization.py:130``). Pinned by F5: start/end are rounded from
    double, step = fl32((end-start)/(n-1)), and element i is a single-rounding
    fma: fma(step, i, start) for i < n//2, fma(-step, n-1-i, end) otherwise."""
    mx = _f32(mx)
    s = _f32(0.2 * float(mx))
    e = _f32(1.2 * float(mx))
    if n == 1:
        return np.array([s], dtype=F32)
    with np.errstate(invalid="ignore", over="ignore"):
        step = _f32(_f32(e - s) / _f32(n - 1))
        i = np.arange(n, dtype=np.float64)
        half = n // 2
        lo = np.float64(step) * i[:half] + np.float64(s)          # exact in f64, one rounding below
        hi = np.float64(e) - np.float64(step) * (n - 1 - i[half:])
    return np.concatenate([lo, hi]).astype(F32)


def _as_rows(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=F32)
    if x.ndim == 0:
        return x.reshape(1, 1)
    if x.ndim == 1:
        return x.reshape(1, -1)
    return x.reshape(-1, x.shape[-1])


def _quads(rows: np.ndarray) -> np.ndarray:
    r, c = rows.shape
    cp = (c + 3) // 4 * 4
    out = np.zeros((r, cp), dtype=F32)
    out[:, :c] = rows
    return out.reshape(r, cp // 4, 4)


def fixed_point_exponent(mx: np.float32, nquads: int) -> int:
    _, e = np.frexp(np.float64(mx))
    return 56 - int(max(nquads - 1, 0)).bit_length() - 2 * int(e)


def _qround(x, scale, qmax):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.clip(np.rint(x / scale), -qmax, qmax - 1)


def mse_sse_table(x: np.ndarray, bits: int, num_attempts: int = 200):
    """Canonical per-candidate SSE (uint64) and the candidate grid."""
    rows = _as_rows(x)
    qmax = 2 ** (bits - 1)
    den = _f32(2 * qmax - 1)
    with np.errstate(invalid="ignore"):
        mx = _f32(max(abs(rows.min()), abs(rows.max()))) if rows.size else _f32(0)
    grid = candidate_grid(mx, num_attempts)
    quads = _quads(rows)
    nq = quads.shape[0] * quads.shape[1]
    K = fixed_point_exponent(mx, nq)
    sse = np.zeros(num_attempts, dtype=np.uint64)
    for c, t in enumerate(grid):
        scale = _f32(_f32(2.0) * t) / den
        q = _qround(quads, scale, qmax)
        d = quads - (q * scale).astype(F32)
        d2 = (d * d).astype(F32)
        g = ((d2[..., 0] + d2[..., 1]).astype(F32) + (d2[..., 2] + d2[..., 3]).astype(F32)).astype(F32)
        fx = np.floor(g.astype(np.float64) * (2.0 ** K)).astype(np.uint64)
        sse[c] = fx.sum(dtype=np.uint64)
    return sse, grid, mx


def _mse_degenerate(mx) -> bool:
    return not (np.isfinite(mx) and mx > 0)


def quantize_tensor_mse(x: np.ndarray, bits: int, num_attempts: int = 200, return_info=False):
    """``source/quantization.py:118-144`` (200-candidate MSE-minmax search)."""
    x = np.asarray(x, dtype=F32)
    rows = _as_rows(x)
    qmax = 2 ** (bits - 1)
    den = _f32(2 * qmax - 1)
    mx = _f32(max(abs(rows.min()), abs(rows.max()))) if rows.size else _f32(0)
    if _mse_degenerate(mx):
        # torch: zero range => 0/0 or nan candidates => every output element is NaN
        y = np.full(x.shape, np.nan, dtype=F32)
        return (y, dict(index=0, t=np.float32(np.nan), scale=np.float32(np.nan))) if return_info else y
    sse, grid, _ = mse_sse_table(x, bits, num_attempts)
    idx = int(np.argmin(sse))
    t = grid[idx]
    scale = _f32(_f32(2.0) * t) / den
    y = (_qround(x, scale, qmax) * scale).astype(F32)
    if return_info:
        return y, dict(index=idx, t=t, scale=scale, sse=sse)
    return y


def min_max_quantize(x: np.ndarray, bits: int) -> np.ndarray:
    """``source/quantization.py:48-66`` (``tensor_minmax``)."""
    x = np.asarray(x, dtype=F32)
    assert bits >= 1, bits
    with np.errstate(all="ignore"):
        if bits == 1:
            return (np.sign(x) - _f32(1)).astype(F32)
        mn, mxv = x.min(), x.max()
        rng = _f32(mxv - mn)
        r = ((x - mn).astype(F32) / rng).astype(F32)
        n = _f32(2.0 ** bits - 1)
        qi = np.floor((r * n).astype(F32) + _f32(0.5)).astype(F32)
        return ((((qi * rng).astype(F32) / n).astype(F32)) + mn).astype(F32)


def quantize_symmetric(x: np.ndarray, bits: int) -> np.ndarray:
    """``source/quantization.py:91-95`` with tensor statistics (``:36-38``)."""
    x = np.asarray(x, dtype=F32)
    qmax = 2 ** (bits - 1)
    den = _f32(2 * qmax - 1)
    with np.errstate(all="ignore"):
        tmax, tmin = x.max(), x.min()
        m = abs(tmin) if abs(tmin) > tmax else tmax
        scale = _f32(_f32(2.0) * _f32(m)) / den
        # `.to(int)` before the multiply (source/quantization.py:95) matters for non-finite data
        return (_to_i64(_qround(x, scale, qmax)).astype(F32) * scale).astype(F32)


def quantize_affine(x: np.ndarray, bits: int, tmin=None, tmax=None) -> np.ndarray:
    """``source/quantization.py:97-106``."""
    x = np.asarray(x, dtype=F32)
    qmax = 2 ** (bits - 1)
    den = _f32(2 * qmax - 1)
    with np.errstate(all="ignore"):
        if tmin is None or tmax is None:
            tmax, tmin = x.max(), x.min()
        tmin, tmax = _f32(tmin), _f32(tmax)
        scale = _f32(_f32(tmax - tmin) / den)
        ratio = _f32(tmin / scale)
        zp = np.int64(-qmax - _trunc_i32(ratio))
        zp = int(np.clip(zp, -qmax, qmax - 1))
        lv = np.clip(np.rint(x / scale).astype(F32) + _f32(zp), -qmax, qmax - 1)
        lv = _to_i64(lv)
        return ((lv - zp).astype(F32) * scale).astype(F32)


def _trunc_i32(v):
    # torch .int() of a float32 scalar: truncation; NaN/inf -> INT_MIN on x86
    if not np.isfinite(v):
        return np.int64(-2 ** 31)
    return np.int64(np.trunc(v))


def _to_i64(a):
    out = np.where(np.isfinite(a), a, 0).astype(np.int64)
    out[~np.isfinite(a)] = np.iinfo(np.int64).min
    return out


def _trunc_i32_vec(v):
    v = np.asarray(v, dtype=F32)
    out = np.where(np.isfinite(v), np.trunc(np.where(np.isfinite(v), v, 0)), 0).astype(np.int64)
    out[~np.isfinite(v) | (v >= 2.0 ** 31) | (v < -2.0 ** 31)] = -2 ** 31
    return out


def _check_broadcast(shape, nch):
    """torch broadcasting of the (nch,) channel statistics against the tensor's LAST
    dimension (the reference divides the tensor by them as they stand)."""
    last = shape[-1] if len(shape) else 1
    if last != nch and last != 1 and nch != 1:
        raise RuntimeError(f"The size of tensor a ({last}) must match the size of tensor b ({nch}) at "
                           f"non-singleton dimension {max(len(shape) - 1, 0)}")


def quantize_channel(x: np.ndarray, bits: int, qscheme: str, dim: int) -> np.ndarray:
    """``channel_symmetric`` / ``channel_affine`` (``source/quantization.py:29-33, 91-106``):
    max/min of every row of ``unfold(x, dim)`` (``source/utils.py:60-74``), then the
    tensor-scheme arithmetic with those (shape[dim],) statistics broadcast against the
    tensor's last dimension, as torch does (an incompatible size raises RuntimeError)."""
    x = np.asarray(x, dtype=F32)
    nd = x.ndim
    if not -max(nd, 1) <= dim < max(nd, 1):
        raise IndexError(f"Dimension out of range (expected to be in range of [{-max(nd, 1)}, {max(nd, 1) - 1}], "
                         f"but got {dim})")
    d = dim % max(nd, 1)
    u = np.moveaxis(x.reshape(x.shape if nd else (1,)), d, 0)
    u = u.reshape(u.shape[0], -1)
    nch = u.shape[0]
    _check_broadcast(x.shape, nch)
    qmax = 2 ** (bits - 1)
    den = _f32(2 * qmax - 1)
    with np.errstate(all="ignore"):
        tmax = u.max(axis=-1).astype(F32)
        tmin = u.min(axis=-1).astype(F32)
        if qscheme == "channel_symmetric":
            m = np.where(np.abs(tmin) > tmax, np.abs(tmin), tmax).astype(F32)
            scale = ((_f32(2.0) * m).astype(F32) / den).astype(F32)
            lv = np.clip(np.rint((x / scale).astype(F32)), -qmax, qmax - 1)
            return (_to_i64(lv).astype(F32) * scale).astype(F32)
        scale = ((tmax - tmin).astype(F32) / den).astype(F32)
        zp = (-qmax - _trunc_i32_vec((tmin / scale).astype(F32))).astype(np.int64)
        zp = ((zp + 2 ** 31) % 2 ** 32 - 2 ** 31)          # int32 wrap (.int())
        zp = np.clip(zp, -qmax, qmax - 1)
        lv = np.clip((np.rint((x / scale).astype(F32)) + zp.astype(F32)).astype(F32), -qmax, qmax - 1)
        return ((_to_i64(lv) - zp).astype(F32) * scale).astype(F32)


def quantize_tensor(x: np.ndarray, bits: int, qscheme: str, dim=None, **kwargs) -> np.ndarray:
    """Dispatch of ``source/quantization.py:69-115`` (error behaviour included)."""
    if qscheme in ("channel_symmetric", "channel_affine"):
        if dim is None:
            raise TypeError("channel statistics need a mode (reference: unfold(tensor, None))")
        return quantize_channel(x, bits, qscheme, dim)
    if qscheme == "tensor_symmetric":
        return quantize_symmetric(x, bits)
    if qscheme == "tensor_affine":
        return quantize_affine(x, bits, kwargs.get("tmin"), kwargs.get("tmax"))
    if qscheme == "tensor_mseminmax_symmetric":
        return quantize_tensor_mse(x, bits, **kwargs)
    if qscheme == "tensor_minmax":
        return min_max_quantize(x, bits)
    raise NotImplementedError(qscheme)
