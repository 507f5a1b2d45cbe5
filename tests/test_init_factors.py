"""init_factors (source/admm.py:21-48) against the reference's own factors (F2), on the
CPU (init is plain torch in both): 'random' bit-exact, 'svd' up to column signs with the
random completion columns bit-exact. The GPU run is tests/test_gpu_reference.py."""
import os

import numpy as np
import pytest
import torch

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


def test_random_init_matches_reference():
    from admmq import init_factors
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    fs = init_factors(torch.from_numpy(z["l1_W"]), rank=134, init="random", device="cpu", seed=42)
    for k, f in zip("ABC", fs):
        assert np.array_equal(f.numpy(), z["l1_" + k])
    fs = init_factors(torch.from_numpy(z["w2_W"]), rank=13, init="random", device="cpu", seed=42)
    assert np.array_equal(fs[0].numpy(), z["w2_A"]) and np.array_equal(fs[1].numpy(), z["w2_B"])


@pytest.mark.parametrize("name,R", [("l1", 134), ("w2", 13)])
def test_svd_init_matches_reference(name, R):
    from admmq import init_factors
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    T = torch.from_numpy(z[f"{name}_W"])
    fs = init_factors(T, rank=R, init="svd", device="cpu", seed=42)
    for m, f in enumerate(fs):
        ref = z[f"{name}_svd_m{m}"]
        got = f.numpy()
        assert got.shape == ref.shape
        ns = min(T.shape[m], R)
        for j in range(ns):
            sgn = np.sign(np.dot(got[:, j], ref[:, j])) or 1.0
            assert _rel(sgn * got[:, j], ref[:, j]) < 1e-4, (m, j)
        assert np.array_equal(got[:, ns:], ref[:, ns:]), m


def test_unknown_init_raises():
    from admmq import init_factors
    with pytest.raises(NotImplementedError):
        init_factors(torch.zeros(4, 5, 6), rank=3, init="bogus", seed=1)
