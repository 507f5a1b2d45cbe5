"""The numpy restatement of scripts/factorize_lowrank.py (oracle/lowrank_oracle.py) against
the reference's own outputs (tests/golden/f6_lowrank.npz, made by gen_golden.py --only f6)."""
import os
from functools import partial

import numpy as np
import pytest

from oracle import lowrank_oracle as lo
from oracle import quant_oracle as qo

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def f6():
    return np.load(os.path.join(GOLDEN, "f6_lowrank.npz"))


def _rel(a, b):
    return float(np.linalg.norm(np.float64(a) - np.float64(b)) / np.linalg.norm(np.float64(b)))


@pytest.mark.parametrize("qs", ["tensor_minmax", "tensor_mseminmax_symmetric"])
@pytest.mark.parametrize("mi", [2, 3, 50])
def test_quant_side_bit_exact(f6, qs, mi):
    """Elementwise float32 updates + the bit-exact quantizer: identical to the reference."""
    qf = partial(qo.quantize_tensor, bits=4, qscheme=qs)
    H, U, _ = lo.admm_iteration(f6["Wq0"], np.zeros_like(f6["Wq0"]), f6["W"], f6["Wr0"], qf, 1.0, mi)
    assert np.array_equal(H.view(np.uint32), f6[f"{qs}_q_it{mi}_H"].view(np.uint32))
    assert np.array_equal(U.view(np.uint32), f6[f"{qs}_q_it{mi}_U"].view(np.uint32))


@pytest.mark.parametrize("mi", [2, 3])
def test_rank_side(f6, mi):
    """SVD truncation (numpy LAPACK vs torch's): within 1e-5 rel-Frobenius."""
    pf = partial(lo.project_rank, rank=4)
    H, U, _ = lo.admm_iteration(f6["Wr0"], np.zeros_like(f6["Wr0"]), f6["W"], f6["Wq0"], pf, 1.0, mi)
    assert _rel(H, f6[f"r_it{mi}_H"]) < 1e-5
    assert _rel(U, f6[f"r_it{mi}_U"]) < 1e-5
    assert np.linalg.matrix_rank(H.astype(np.float64), tol=1e-4 * np.linalg.norm(H)) <= 4
