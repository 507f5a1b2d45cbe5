"""The CPU oracle of the CP-ALS and CP-EPC initialisers (oracle/epc_oracle.py; the
product admmq.parafac_epc runs the same algorithm on the fp64 HIP contractions and is
checked against this oracle in tests/test_gpu_epc.py). source/parafac_epc.py:12-82.

Parity unpinned (tensorly / musco-pytorch absent offline): these are
objective-level checks of the published algorithms - the EPC result keeps the ALS
reconstruction error (||Y - [[lambda; U]]|| <= delta) while not increasing the
intensities ||lambda||, with unit-norm factor columns and the reference's return layout."""
import pytest
import torch

from oracle.epc_oracle import _reconstruct, cp_anc, parafac, parafac_epc


def _lowrank(shape, R, noise, seed):
    g = torch.Generator().manual_seed(seed)
    fs = [torch.randn(n, R, generator=g, dtype=torch.float64) for n in shape]
    Y = _reconstruct(None, fs)
    return Y + noise * torch.randn(*shape, generator=g, dtype=torch.float64) * Y.norm() / Y.numel() ** 0.5


def test_parafac_recovers_exact_low_rank():
    Y = _lowrank((7, 6, 5), 3, 0.0, 0)
    w, fs = parafac(Y, 3, random_state=1, tol=1e-14, n_iter_max=2000, normalize_factors=True)
    rel = float((Y - _reconstruct(w, fs)).norm() / Y.norm())
    assert rel < 1e-6
    for f in fs:
        torch.testing.assert_close(f.norm(dim=0), torch.ones(3, dtype=torch.float64))


def test_cp_anc_keeps_error_and_lowers_intensities():
    Y = _lowrank((9, 8, 6), 6, 0.3, 2)       # over-parameterised: ALS intensities can blow up
    w, fs = parafac(Y, 6, random_state=3, tol=1e-10, n_iter_max=500, normalize_factors=True)
    delta = float((Y - _reconstruct(w, fs)).norm())
    w2, fs2 = cp_anc(Y, 6, delta, w, fs, maxiter=200, tol=1e-9)
    err = float((Y - _reconstruct(w2, fs2)).norm())
    assert err <= delta * (1 + 1e-6)
    assert float(w2.norm()) <= float(w.norm()) * (1 + 1e-9)
    for f in fs2:
        torch.testing.assert_close(f.norm(dim=0), torch.ones(6, dtype=torch.float64))


def test_parafac_epc_layout_and_objective():
    Y = _lowrank((10, 4, 9), 5, 0.2, 4)      # modes unsorted: the driver permutes and restores
    lam, Us = parafac_epc(Y, 5, als_maxiter=300, epc_maxiter=50, epc_rounds=5)
    assert [tuple(u.shape) for u in Us] == [(10, 5), (4, 5), (9, 5)]
    assert lam.shape == (5,) and bool((lam > 0).all())
    order = sorted(range(3), key=lambda m: Y.shape[m])
    w, fs = parafac(Y.permute(*order), 5, tol=1e-5, n_iter_max=300, normalize_factors=True)
    als_err = float((Y.permute(*order) - _reconstruct(w, fs)).norm())
    epc_err = float((Y - _reconstruct(lam, Us)).norm())
    assert epc_err <= als_err * (1 + 1e-6)
    assert float(lam.norm()) <= float(w.norm()) * (1 + 1e-9)


def test_product_has_no_cpu_path():
    """admmq.parafac_epc is the HIP product: a CPU tensor raises instead of running on the host."""
    from admmq import parafac_epc as product
    with pytest.raises(RuntimeError):
        product.parafac(torch.zeros(3, 4, 5, dtype=torch.float64), 2, n_iter_max=1)
