"""ORACLE — test infrastructure only. ctypes binding of quant_oracle_c.c (the C
restatement of :mod:`oracle.quant_oracle`, for full-size parity checks).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s parity leg use it.
The library is built by ``__graft_entry__.build()`` (``make -C oracle``); when it is
missing (a fresh tree) it is compiled here with gcc on first use.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libquant_oracle.so")
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(_HERE, "quant_oracle_c.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    lib = ctypes.CDLL(_SO)
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    lib.oq_sse_table.restype = I32
    lib.oq_sse_table.argtypes = [P, I64, I64, I32, I32, P, P, P]
    lib.oq_argmin.restype = I32
    lib.oq_argmin.argtypes = [P, I32, I32, I32, I64]
    lib.oq_quantize_mse.restype = I32
    lib.oq_quantize_mse.argtypes = [P, I64, I64, I32, I32, I32, P]
    lib.oq_absmax.restype = ctypes.c_float
    lib.oq_absmax.argtypes = [P, I64]
    _lib = lib
    return lib


def _rows(x):
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if x.ndim == 0:
        return x.reshape(1, 1)
    if x.ndim == 1:
        return x.reshape(1, -1)
    return x.reshape(-1, x.shape[-1])


def sse_table(x, bits, num_attempts=200):
    """(sse uint64[num_attempts], grid float32[num_attempts], mx, K) - same table as
    quant_oracle.mse_sse_table."""
    r = _rows(x)
    sse = np.zeros(num_attempts, np.uint64)
    grid = np.zeros(num_attempts, np.float32)
    mx = ctypes.c_float(0)
    K = load().oq_sse_table(r.ctypes.data, r.shape[0], r.shape[1], bits, num_attempts, sse.ctypes.data,
                            grid.ctypes.data, ctypes.byref(mx))
    return sse, grid, np.float32(mx.value), int(K)


def argmin(sse, rule, K, nelem):
    sse = np.ascontiguousarray(sse, np.uint64)
    return int(load().oq_argmin(sse.ctypes.data, len(sse), int(rule), int(K), int(nelem)))


def rule1_means(sse, K, nelem):
    """The float32 means of rule 1 (fl32(fl32(S) / fl32(n)), S = sse 2^-K)."""
    s = np.ldexp(np.asarray(sse, np.uint64).astype(np.float32).astype(np.float64), -K).astype(np.float32)
    return (s / np.float32(nelem)).astype(np.float32)


def quantize_mse(x, bits, num_attempts=200, rule=0):
    """(y, index): quantize_tensor_mse under the given argmin rule."""
    x = np.asarray(x, dtype=np.float32)
    r = _rows(x)
    y = np.empty_like(r)
    idx = load().oq_quantize_mse(r.ctypes.data, r.shape[0], r.shape[1], bits, num_attempts, int(rule), y.ctypes.data)
    return y.reshape(x.shape), int(idx)
