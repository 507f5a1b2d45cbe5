"""CPU check of the two-stage MSE search math (oracle/stage1_model.py): the bound E(c)
really encloses the canonical SSE, and the candidate set S always contains the
oracle's brute-force first-index argmin (and is usually a single candidate)."""
import numpy as np
import pytest

import golden_cases as gc
from oracle import quant_oracle as qo
from oracle import stage1_model as sm


def _check(x, bits, n=200):
    sse, grid, mx = qo.mse_sse_table(x, bits, n)
    S, A, E, K = sm.candidate_set(x, bits, n)
    exact = sse.astype(np.float64) * 2.0 ** (-K)
    assert np.all(np.abs(exact - A) <= E), np.max(np.abs(exact - A) / E)
    best = int(np.argmin(sse))
    assert best in S
    return len(S)


@pytest.mark.parametrize("seed", range(12))
def test_bound_and_set(seed):
    rng = np.random.default_rng(seed)
    shape = [(9, 134), (64, 134), (37, 53), (128, 50)][seed % 4]
    bits = [4, 2, 3, 8][(seed // 4) % 4]
    scale = [1.0, 1e-3, 0.3][seed % 3]
    x = (rng.standard_normal(shape) * scale).astype(np.float32)
    if seed % 5 == 0:
        x[0, 0] = 25 * scale     # outlier
    assert _check(x, bits) <= 3


def test_edge_kats():
    sizes = []
    for case in gc.f1_cases():
        if case["qscheme"] != "tensor_mseminmax_symmetric" or case["kind"] in ("zeros", "nan", "inf"):
            continue
        if np.prod(case["shape"]) > 20000:
            continue
        x = gc.f1_input(case)
        sizes.append(_check(x, case["bits"], case.get("num_attempts") or 200))
    assert max(sizes) >= 1
