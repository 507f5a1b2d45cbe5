"""fp64 HIP contractions of the CP-ALS / EPC initialiser (csrc/cp64_kernels.hip via
admmq.als.gram_mttkrp_f64) and admmq.parafac_epc on them, against the CPU oracle
(oracle/epc_oracle.py, fp64 torch). source/parafac_epc.py:12-82.

Parity unpinned against the reference itself (tensorly / musco absent offline): the
contractions are checked against fp64 einsum (1e-12 relative: fp64 with another
summation order), the drivers against the oracle's run of the same algorithm from the
same random start (agreement to fp64 rounding drift, 1e-6 on the factors)."""
import time

import numpy as np
import pytest
import torch

from conftest import gpu_available
from oracle import epc_oracle as eo

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


@pytest.mark.parametrize("shape,R", [((7, 6, 5), 3), ((64, 64, 9), 134), ((9, 64, 64), 134), ((128, 64, 9), 183),
                                     ((512, 512, 9), 1141), ((64, 48), 13), ((300, 2048), 200), ((1, 17, 3), 40)])
def test_cp64_gram_mttkrp_vs_einsum(shape, R):
    from admmq.als import gram_mttkrp_f64
    g = torch.Generator().manual_seed(sum(shape) + R)
    Y = torch.randn(*shape, generator=g, dtype=torch.float64)
    fs = [torch.randn(n, R, generator=g, dtype=torch.float64) for n in shape]
    dev = torch.device("cuda:0")
    for mode in range(len(shape)):
        F, G = gram_mttkrp_f64(Y.to(dev), [f.to(dev) for f in fs], mode)
        Fo, Go = eo._mttkrp_gram(Y, fs, mode)
        assert _rel(F, Fo) < 1e-12, (shape, mode, _rel(F, Fo))
        assert _rel(G, Go) < 1e-12, (shape, mode, _rel(G, Go))


def _lowrank(shape, R, noise, seed):
    g = torch.Generator().manual_seed(seed)
    fs = [torch.randn(n, R, generator=g, dtype=torch.float64) for n in shape]
    Y = eo._reconstruct(None, fs)
    return Y + noise * torch.randn(*shape, generator=g, dtype=torch.float64) * Y.norm() / Y.numel() ** 0.5


def test_parafac_matches_oracle():
    from admmq import parafac_epc as pe
    Y = _lowrank((10, 8, 9), 4, 0.1, 7)
    w, fs = pe.parafac(Y.cuda(), 4, random_state=2, tol=1e-12, n_iter_max=30, normalize_factors=True)
    wo, fso = eo.parafac(Y, 4, random_state=2, tol=1e-12, n_iter_max=30, normalize_factors=True)
    assert _rel(w, wo) < 1e-6
    for f, fo in zip(fs, fso):
        assert _rel(f, fo) < 1e-6
    rel = float((Y - eo._reconstruct(w.cpu(), [f.cpu() for f in fs])).norm() / Y.norm())
    assert rel < 0.2


def test_cp_anc_and_parafac_epc_match_oracle():
    from admmq import parafac_epc as pe
    Y = _lowrank((9, 8, 6), 6, 0.3, 2)       # over-parameterised: ALS intensities can blow up
    w, fs = eo.parafac(Y, 6, random_state=3, tol=1e-10, n_iter_max=200, normalize_factors=True)
    delta = float((Y - eo._reconstruct(w, fs)).norm())
    w2, fs2 = pe.cp_anc(Y.cuda(), 6, delta, w.cuda(), [f.cuda() for f in fs], maxiter=100, tol=1e-9)
    w2o, fs2o = eo.cp_anc(Y, 6, delta, w, fs, maxiter=100, tol=1e-9)
    err = float((Y - eo._reconstruct(w2.cpu(), [f.cpu() for f in fs2])).norm())
    assert err <= delta * (1 + 1e-6)
    assert float(w2.norm()) <= float(w.norm()) * (1 + 1e-9)
    assert _rel(w2, w2o) < 1e-6
    Y3 = _lowrank((10, 4, 9), 5, 0.2, 4)     # modes unsorted: the driver permutes and restores
    lam, Us = pe.parafac_epc(Y3.cuda(), 5, als_maxiter=100, epc_maxiter=30, epc_rounds=3)
    lamo, Uso = eo.parafac_epc(Y3, 5, als_maxiter=100, epc_maxiter=30, epc_rounds=3)
    assert [tuple(u.shape) for u in Us] == [(10, 5), (4, 5), (9, 5)]
    assert _rel(lam, lamo) < 1e-6
    for u, uo in zip(Us, Uso):
        assert _rel(u, uo) < 1e-6


def test_parafac_epc_resnet18_layer_timing():
    """init_factors('parafac-epc')'s call (50 ALS + 50 EPC iterations per round,
    source/admm.py:40-44) on layer1.0.conv1 (64, 64, 9), R = 134: runs on the device,
    keeps the ALS error (EPC), reports its wall time."""
    from admmq import synthetic
    from admmq.parafac_epc import parafac, parafac_epc
    idx, spec = synthetic.find_layer("resnet18", "layer1.0.conv1")
    W = torch.from_numpy(synthetic.layer_weight(spec, idx)).cuda().double()
    R = spec.rank()
    torch.cuda.synchronize()
    t0 = time.time()
    lam, Us = parafac_epc(W, R, als_maxiter=50, epc_maxiter=50)
    torch.cuda.synchronize()
    t = time.time() - t0
    w, fs = parafac(W, R, tol=1e-5, n_iter_max=50, normalize_factors=True)
    als_err = float((W - eo._reconstruct(w, fs)).norm() / W.norm())
    epc_err = float((W - eo._reconstruct(lam, Us)).norm() / W.norm())
    print(f"parafac-epc layer1.0.conv1 R={R}: {t:.2f} s, ALS rel err {als_err:.4f}, EPC rel err {epc_err:.4f}")
    assert np.isfinite(epc_err) and epc_err <= als_err * (1 + 1e-6)


@pytest.mark.parametrize("R,seed", [(134, 1), (13, 2), (1141, 3), (5, 4)])
def test_epc_mu_device_matches_oracle(R, seed):
    """The EPC multiplier solved on the device (admmq_epc_mu: bracket doubling + bisection to
    fp64 resolution, one workgroup) against the oracle's host restatement of the same root
    search: within a few ulps of the bracket (the sum over the R terms runs in another
    order); 0 when the unconstrained step already meets delta."""
    from admmq import panel
    g = torch.Generator().manual_seed(seed)
    s = torch.rand(R, generator=g, dtype=torch.float64) * 10.0
    s[0] = 0.0   # a zero eigenvalue (clamped) as cp_anc can see
    c = torch.rand(R, generator=g, dtype=torch.float64)
    normY2 = float(torch.sum(c / s.clamp_min(1e-3))) * 2.0
    for delta2 in (normY2 * 0.5, normY2 * 0.999, normY2 * 2.0):
        ref = eo._solve_mu(c, s, normY2, delta2)
        got = float(panel.epc_mu(c.cuda(), s.cuda(), normY2, delta2))
        assert abs(got - ref) <= 1e-12 * max(abs(ref), 1e-300) or (ref == 0.0 and got == 0.0), (delta2, got, ref)


@pytest.mark.parametrize("n,m", [(1, 3), (5, 9), (64, 1), (134, 64), (134, 9), (136, 130)])
def test_spd_solve64_vs_library(n, m):
    """The one-workgroup fp64 solve (csrc/epc_kernels.hip: Gauss-Jordan inverse in LDS,
    16-lane substitution groups) that replaces tensorly parafac's torch.linalg.solve
    (source/parafac_epc.py:42): X = F G^-1 within 1e-11 of the float64 library solve on a
    well-conditioned SPD G, at n up to the LDS limit and m above one pass of 64 rows."""
    from admmq import panel
    g = torch.Generator().manual_seed(n * 1000 + m)
    B = torch.randn(n, 2 * n + 3, generator=g, dtype=torch.float64)
    G = B @ B.T / (2 * n + 3) + 0.1 * torch.eye(n, dtype=torch.float64)
    F = torch.randn(m, n, generator=g, dtype=torch.float64)
    X = panel.spd_solve64(G.cuda(), F.cuda())
    ref = torch.linalg.solve(G, F.T).T
    assert _rel(X, ref) < 1e-11, _rel(X, ref)


@pytest.mark.parametrize("n,m,seed", [(134, 64, 1), (134, 9, 2), (7, 5, 3), (136, 64, 4), (1, 3, 5), (2, 7, 6),
                                      (3, 70, 7), (40, 200, 8), (136, 1100, 9)])
def test_epc_step64_vs_eigen_form(n, m, seed):
    """The EPC mode update on the device (csrc/epc_kernels.hip: G tridiagonalised once,
    safeguarded Newton on tridiagonal L D L^T recurrences, no eigendecomposition) against
    the eigen form the oracle uses (oracle/epc_oracle.py: eigh, mu by bisection to fp64
    resolution, U = F V diag(1/(s + mu)) V^T) in float64 on the CPU: mu and U within 1e-9,
    for targets needing mu > 0 (with and without a warm start) and for one the
    least-squares step already meets (mu = 0). Sizes: no reflector (n = 1, 2), one
    (n = 3), the LDS limit (136), several 64-row passes of the reflector products
    (m = 70, 200) and more rows than threads (m = 1100)."""
    from admmq import panel
    g = torch.Generator().manual_seed(seed)
    B = torch.randn(n, n + 8, generator=g, dtype=torch.float64)
    G = B @ B.T / (n + 8) + 1e-3 * torch.eye(n, dtype=torch.float64)
    F = torch.randn(m, n, generator=g, dtype=torch.float64)
    s, V = torch.linalg.eigh(G)
    s = s.clamp_min(0.0)
    Ft = F @ V
    c = torch.sum(Ft * Ft, dim=0)
    ls = float(torch.sum(c / s))            # <F, F G^-1>: e(0) = normY2 - ls
    normY2 = ls * 1.5
    e0 = normY2 - ls
    # (normY2 = 3 e0, so delta2 < normY2: a finite root)
    for delta2, warm in ((e0 * 1.5, 0.0), (e0 * 2.5, 0.0), (e0 * 2.5, 0.37 * float(s.mean())), (e0 * 0.5, 0.0)):
        ref_mu = eo._solve_mu(c, s, normY2, delta2)
        ref_X = (Ft / (s + ref_mu).clamp_min(1e-300)) @ V.T
        mu = torch.tensor(warm, dtype=torch.float64, device="cuda")
        X = panel.epc_step64(G.cuda(), F.cuda(), normY2, delta2, mu)
        got = float(mu)
        if ref_mu == 0.0:
            assert got == 0.0
        else:
            assert abs(got - ref_mu) <= 1e-8 * ref_mu, (delta2, warm, got, ref_mu)
        assert _rel(X, ref_X) < 1e-9, (delta2, warm, _rel(X, ref_X))


@pytest.mark.parametrize("rows,R", [((9, 64), 134), ((512, 512), 1141), ((7, None), 5)])
def test_colnorm64_vs_torch(rows, R):
    """The one-launch normalisation of cp_anc's other factors (admmq_cp_colnorm64) against
    torch's U / norm(U, dim=0).clamp_min(1e-300): within 1e-15 relative (another summation
    order of the column norms), a zero column left at zero, inputs untouched."""
    from admmq import panel
    g = torch.Generator().manual_seed(R)
    A = torch.randn(rows[0], R, generator=g, dtype=torch.float64)
    A[:, 0] = 0.0
    B = torch.randn(rows[1], R, generator=g, dtype=torch.float64) if rows[1] else None
    Ad, Bd = A.cuda(), (B.cuda() if B is not None else None)
    oA, oB = panel.colnorm64(Ad, Bd)
    for src, out in ((A, oA), (B, oB)):
        if src is None:
            assert out is None
            continue
        ref = src / torch.linalg.norm(src, dim=0).clamp_min(1e-300)
        assert _rel(out, ref) < 1e-15, _rel(out, ref)
    assert float(oA[:, 0].abs().max()) == 0.0
    assert torch.equal(Ad.cpu(), A)
