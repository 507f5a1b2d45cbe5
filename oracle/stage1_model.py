"""ORACLE — test infrastructure only. numpy model of the two-stage exact MSE search
that the HIP kernels implement (k_hist_admm / k_select_admm / k_sse_sel_admm).

Stage 1 computes, per candidate c, the exact-arithmetic SSE through per-element level
breakpoints:  SSE_e(c) = S2 - 2 s_c T1(c) + s_c^2 T2(c), with T1 = sum |q||x| and
T2 = sum q^2 over the clamped levels q = clamp(rint(fl(x/s_c))). A rigorous bound
E(c) >= |SSE_canon(c) 2^-K - SSE_e(c)| (float32 roundings of the canonical rule,
the fixed-point floor and float64 accumulation) gives the candidate set
S = {c : A(c) - E(c) <= min_c' A(c') + E(c')}, which provably contains the canonical
first-index argmin. Stage 2 evaluates the canonical SSE only on S.

This file exists so the bound logic is checked on CPU (tests/test_stage1_model.py)
against the oracle's brute-force argmin; it mirrors csrc/quant_device.h.
"""
from __future__ import annotations

import numpy as np

from . import quant_oracle as qo

U = 2.0 ** -24


def levels(a: np.ndarray, s: np.float32, cap: np.ndarray) -> np.ndarray:
    """|q| = min(rint(fl(a/s)), cap) with IEEE float32 division (a >= 0)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.minimum(np.rint((a / s).astype(np.float32)), cap)


def stage1_tables(x: np.ndarray, bits: int, n: int = 200, K1_bits: int = 0):
    rows = qo._as_rows(x)
    flat = rows.reshape(-1)
    qmax = 2 ** (bits - 1)
    den = np.float32(2 * qmax - 1)
    mx = np.float32(max(abs(rows.min()), abs(rows.max())))
    grid = qo.candidate_grid(mx, n)
    scales = (np.float32(2.0) * grid / den).astype(np.float32)
    a = np.abs(flat).astype(np.float32)
    cap = np.where(flat > 0, qmax - 1, qmax).astype(np.float32)
    # per (element, level k) breakpoint b = #{c : level(c) >= k}; histogram form
    T1 = np.zeros(n)
    T2 = np.zeros(n)
    for c in range(n):                   # (model: direct per-candidate evaluation; the GPU
        lv = levels(a, scales[c], cap)   #  builds the same sums from breakpoints)
        T1[c] = float(np.sum(lv.astype(np.float64) * a.astype(np.float64)))
        T2[c] = float(np.sum(lv.astype(np.float64) ** 2))
    S2 = float(np.sum(flat.astype(np.float64) ** 2))
    return dict(mx=mx, grid=grid, scales=scales, T1=T1, T2=T2, S2=S2, N=flat.size)


def bounds(tab, nq: int, K: int, nterms_fix: int = 0, K1: int = 60):
    """E(c): float32 roundings (relative), float32 underflow (absolute, 8 N 2^-149),
    the canonical floor (nq 2^-K), fixed-point T1 truncation and float64 slack."""
    s = tab["scales"].astype(np.float64)
    T1, T2, S2 = tab["T1"], tab["T2"], tab["S2"]
    A = S2 - 2.0 * s * T1 + s * s * T2
    mag = S2 + 2.0 * s * T1 + s * s * T2
    slack64 = 1e-10 * mag
    SSEhi = np.maximum(A, 0.0) + slack64
    B1 = 2 * U * (1 + U) * (s * np.sqrt(T2 * SSEhi) + SSEhi) + 2 * U * U * (1 + U) ** 2 * (s * s * T2 + SSEhi)
    E = (B1 + 3.0000002 * U * (SSEhi + B1) + nq * 2.0 ** (-K) + 2.0 * s * nterms_fix * 2.0 ** (-K1) + slack64
         + 8.0 * tab["N"] * 2.0 ** -149)
    return A, E


def candidate_set(x: np.ndarray, bits: int, n: int = 200):
    tab = stage1_tables(x, bits, n)
    rows = qo._as_rows(x)
    nq = rows.shape[0] * ((rows.shape[1] + 3) // 4)
    K = qo.fixed_point_exponent(tab["mx"], nq)
    A, E = bounds(tab, nq, K)
    best_hi = np.min(A + E)
    S = np.nonzero(A - E <= best_hi)[0]
    return S, A, E, K
