"""Case tables shared by the golden generator and the parity tests.

Inputs are regenerated from numpy seeds (PCG64 is platform-independent), so the
fixtures only hold reference *outputs* (arrays for small cases, SHA-256 digests
for the rest).
"""
from __future__ import annotations

import hashlib

import numpy as np

F1_SHAPES = [(9, 134), (64, 134), (9, 1141), (128, 278)]
F1_SCALES = [1e-3, 0.05, 1.0]
F1_BITS = [2, 3, 4, 8]
F1_SCHEMES = ["tensor_mseminmax_symmetric", "tensor_minmax", "tensor_symmetric", "tensor_affine"]
F2_SCHEMES = ["tensor_mseminmax_symmetric", "tensor_minmax", "tensor_symmetric", "tensor_affine"]


def f1_cases():
    cases = []
    seed = 0
    for shape in F1_SHAPES:
        for scale in F1_SCALES:
            for bits in F1_BITS:
                for qs in F1_SCHEMES:
                    seed += 1
                    cases.append(dict(id=f"c{seed:04d}", kind="randn", shape=list(shape), scale=scale,
                                      bits=bits, qscheme=qs, seed=seed, num_attempts=None,
                                      store=shape == (9, 134)))
    # large MSE-minmax shapes (digest only): layer4-sized factor, Llama-ish wide row
    for shape, bits in (((512, 1141), 4), ((256, 566), 4), ((64, 1492), 2)):
        seed += 1
        cases.append(dict(id=f"c{seed:04d}", kind="randn", shape=list(shape), scale=0.3, bits=bits,
                          qscheme="tensor_mseminmax_symmetric", seed=seed, num_attempts=None, store=False))
    # num_attempts variants (scripts/custom_benchmark.py:195 uses 1000)
    for na in (1000, 50, 7, 2, 1):
        seed += 1
        cases.append(dict(id=f"c{seed:04d}", kind="randn", shape=[64, 134], scale=1.0, bits=4,
                          qscheme="tensor_mseminmax_symmetric", seed=seed, num_attempts=na, store=True))
    # edge cases
    edge = [
        ("zeros", [9, 134]), ("const", [3, 5]), ("one", [1, 1]), ("vec", [7]), ("cube", [2, 3, 4]),
        ("outlier", [16, 40]), ("negative", [8, 13]), ("ints", [6, 20]), ("nan", [4, 9]), ("inf", [4, 9]),
        ("tiny", [5, 17]), ("halfgrid", [8, 33]), ("bits1", [9, 134]),
    ]
    for kind, shape in edge:
        for qs in F1_SCHEMES:
            seed += 1
            cases.append(dict(id=f"c{seed:04d}", kind=kind, shape=shape, scale=1.0,
                              bits=1 if kind == "bits1" else 4, qscheme=qs, seed=seed,
                              num_attempts=None, store=True))
    # error behaviour (source/quantization.py:29-41, 114-115)
    for qs in ("channel_symmetric", "channel_affine", "tensor_log", "bogus"):
        seed += 1
        cases.append(dict(id=f"c{seed:04d}", kind="randn", shape=[4, 6], scale=1.0, bits=4, qscheme=qs,
                          seed=seed, num_attempts=None, store=False))
    return cases


def f1_input(case) -> np.ndarray:
    shape = tuple(case["shape"])
    rng = np.random.default_rng(case["seed"])
    kind = case["kind"]
    if kind in ("randn", "bits1"):
        x = rng.standard_normal(shape) * case["scale"]
    elif kind == "zeros":
        x = np.zeros(shape)
    elif kind == "const":
        x = np.full(shape, 0.5)
    elif kind == "one":
        x = np.full(shape, -1.25)
    elif kind in ("vec", "cube"):
        x = rng.standard_normal(shape)
    elif kind == "outlier":
        x = rng.standard_normal(shape) * 0.01
        x.flat[17] = 3.0
    elif kind == "negative":
        x = -np.abs(rng.standard_normal(shape)) - 0.1
    elif kind == "ints":
        x = rng.integers(-9, 9, shape).astype(np.float64)
    elif kind == "nan":
        x = rng.standard_normal(shape)
        x.flat[3] = np.nan
    elif kind == "inf":
        x = rng.standard_normal(shape)
        x.flat[5] = np.inf
    elif kind == "tiny":
        x = rng.standard_normal(shape) * 1e-30
    elif kind == "halfgrid":
        # values on k/2 multiples of a candidate-like scale: exercises round-half-even
        x = rng.integers(-16, 16, shape) * 0.5 * (2.0 * 0.6 / 15.0)
    else:
        raise ValueError(kind)
    return x.astype(np.float32)


def canonical_sha(a) -> str:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32)).copy()
    a[np.isnan(a)] = np.float32(np.nan)
    u = a.view(np.uint32)
    u[np.isnan(a)] = np.uint32(0x7FC00000)
    return hashlib.sha256(u.tobytes()).hexdigest()


def grid_levels(H):
    """(levels, scale) of a tensor on a uniform quantization grid: H = fl32(k * s) with
    integer k. s is the smallest positive |H| (some element has |k| = 1 on every real
    factor; checked: every element must then reproduce as k * s)."""
    H = np.asarray(H, np.float32)
    a = np.abs(H[np.isfinite(H)])
    pos = a[a > 0]
    if pos.size == 0:
        return np.zeros(H.shape, np.int64), np.float32(0)
    s = np.float32(pos.min())
    k = np.rint(H.astype(np.float64) / np.float64(s))
    if not np.array_equal((k.astype(np.float32) * s).astype(np.float32), H):
        return None, s
    return k.astype(np.int64), s


def level_mismatch(H, H_ref, X, half_window=1e-4):
    """P2 of SURVEY §8(c): compare the integer levels of two quantized factors.
    Returns (n_mismatch, n_unexplained): mismatches, and those NOT explained by a
    near-half rounding of X (|X/s - (k + 1/2)| < half_window with our own scale s),
    or None when either tensor is not on a uniform grid (the scheme is affine)."""
    k, s = grid_levels(H)
    kr, sr = grid_levels(H_ref)
    if k is None or kr is None:
        return None
    bad = k != kr
    y = np.asarray(X, np.float64) / np.float64(s)
    near = np.abs(np.abs(y - np.floor(y)) - 0.5) < half_window
    return int(bad.sum()), int((bad & ~(near & (np.abs(k - kr) == 1))).sum())


# F9: per-channel quantizers with an explicit dim (source/quantization.py:29-33, 91-106).
# The per-channel stats (shape (shape[dim],)) broadcast against the tensor's LAST dimension
# (torch broadcasting), so a dim other than the last works only when the sizes agree (or
# one is 1) - otherwise the reference raises RuntimeError. Kept as the reference does it.
F9_LAYOUTS = [
    ((64, 134), 1), ((64, 134), 0), ((64, 64), 0), ((16, 8, 9), 2), ((9, 8, 9), 0), ((5, 1), 0),
    ((100,), 0), ((16, 8, 9), -1), ((7, 3, 4), 1), ((1, 1), 0), ((1, 1), 1), ((12, 1, 3), 1),
]


def f9_cases():
    cases = []
    seed = 9000
    for shape, dim in F9_LAYOUTS:
        for qs in ("channel_symmetric", "channel_affine"):
            for bits, scale in ((4, 1.0), (2, 1e-3), (8, 0.05)):
                seed += 1
                cases.append(dict(id=f"k{seed:05d}", kind="randn", shape=list(shape), dim=dim, scale=scale,
                                  bits=bits, qscheme=qs, seed=seed))
    # constant / zero / NaN / inf channels (scale 0, NaN stats; torch's x86 conversions)
    for kind in ("constcol", "nancol", "infcol"):
        for qs in ("channel_symmetric", "channel_affine"):
            seed += 1
            cases.append(dict(id=f"k{seed:05d}", kind=kind, shape=[6, 10], dim=1, scale=1.0, bits=4, qscheme=qs,
                              seed=seed))
    return cases


def f9_input(case) -> np.ndarray:
    shape = tuple(case["shape"])
    rng = np.random.default_rng(case["seed"])
    x = rng.standard_normal(shape) * case["scale"]
    if case["kind"] == "constcol":
        x[:, 3] = 0.75
        x[:, 6] = 0.0
    elif case["kind"] == "nancol":
        x[2, 4] = np.nan
    elif case["kind"] == "infcol":
        x[1, 7] = np.inf
        x[4, 2] = -np.inf
    return x.astype(np.float32)
