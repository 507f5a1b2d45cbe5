"""The CP-ALS / EPC initialiser's R x R solves at every resnet rank (csrc/solve64.hip: the
blocked fp64 Cholesky, L^-1 and fp64-MFMA products spread over the chip; the device-side
multiplier search of epc_search.h), and the drivers of admmq.parafac_epc on them at real
layer sizes. Reference: source/parafac_epc.py:42 (tensorly parafac's torch.linalg.solve) and
:61-74 (musco cp_anc's eigendecomposition + multiplier); both libraries are absent offline, so
the solves are pinned to float64 library solves / the eigen form of oracle/epc_oracle.py on
the CPU, and the drivers to the oracle's run of the same algorithm (parity unpinned against
tensorly / musco themselves)."""
import time

import pytest
import torch

from conftest import gpu_available
from oracle import epc_oracle as eo

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

RANKS = [183, 278, 566, 1141]   # resnet18's 3x3 conv ranks above the one-workgroup limit (136)


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _spd(n, seed, extra=8, ridge=1e-3):
    g = torch.Generator().manual_seed(seed)
    B = torch.randn(n, n + extra, generator=g, dtype=torch.float64)
    return B @ B.T / (n + extra) + ridge * torch.eye(n, dtype=torch.float64), g


@pytest.mark.parametrize("n,m", [(137, 5), (183, 64), (278, 128), (566, 256), (1141, 512), (1141, 9), (1500, 70)])
def test_blocked_spd_solve64_vs_library(n, m):
    """X = F G^-1 by the blocked path within 1e-10 of the float64 library solve, info 0."""
    from admmq import panel
    G, g = _spd(n, n * 7 + m)
    F = torch.randn(m, n, generator=g, dtype=torch.float64)
    info = torch.full((1,), -7, dtype=torch.int32, device="cuda")
    X = panel.spd_solve64(G.cuda(), F.cuda(), info=info)
    ref = torch.linalg.solve(G, F.T).T
    assert int(info) == 0
    assert _rel(X, ref) < 1e-10, _rel(X, ref)


@pytest.mark.parametrize("n", [40, 300])
def test_spd_solve64_reports_indefinite_and_shift_repairs(n):
    """A singular / indefinite G sets info = 1 (small and blocked forms) instead of returning
    garbage silently; the relative shift gives a finite solve of the shifted system."""
    from admmq import panel
    g = torch.Generator().manual_seed(n)
    B = torch.randn(n, n // 2, generator=g, dtype=torch.float64)
    G = B @ B.T                                  # rank n / 2: positive semidefinite, singular
    G[0, 0] -= 1e-3                              # and slightly indefinite
    F = torch.randn(9, n, generator=g, dtype=torch.float64)
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    panel.spd_solve64(G.cuda(), F.cuda(), info=info)
    assert int(info) == 1
    Gs = G + 1e-3 * float(torch.trace(G)) / n * torch.eye(n, dtype=torch.float64)
    if float(torch.linalg.eigvalsh(Gs).min()) > 0:
        X = panel.spd_solve64(G.cuda(), F.cuda(), info=info, rel_shift=1e-3)
        assert int(info) == 0
        assert _rel(X, torch.linalg.solve(Gs, F.T).T) < 1e-8


def _eigen_reference(G, F, normY2, delta2):
    s, V = torch.linalg.eigh(G)
    s = s.clamp_min(0.0)
    Ft = F @ V
    mu = eo._solve_mu(torch.sum(Ft * Ft, dim=0), s, normY2, delta2)
    return mu, (Ft / (s + mu).clamp_min(1e-300)) @ V.T


@pytest.mark.parametrize("n,m", [(134, 64), (183, 64), (278, 128), (566, 256), (1141, 512), (1141, 9)])
def test_blocked_epc_step_vs_eigen_form(n, m):
    """The blocked EPC mode update (a Cholesky of G + mu I per evaluation, the Newton search on
    the device) against the oracle's eigen form (eigh, mu by bisection to fp64 resolution):
    mu within 1e-8 relative and X within 1e-9, for targets needing mu > 0 (cold and warm) and
    one the least-squares step already meets (mu = 0); n = 134 also against the one-workgroup
    tridiagonal kernel."""
    from admmq import panel
    G, g = _spd(n, n + 3 * m)
    F = torch.randn(m, n, generator=g, dtype=torch.float64)
    s, V = torch.linalg.eigh(G)
    Ft = F @ V
    ls = float(torch.sum(torch.sum(Ft * Ft, dim=0) / s))
    normY2 = ls * 1.5
    e0 = normY2 - ls
    Gd, Fd = G.cuda(), F.cuda()
    for delta2, warm in ((e0 * 1.5, 0.0), (e0 * 2.5, 0.0), (e0 * 2.5, 0.37 * float(s.mean())), (e0 * 0.5, 0.0)):
        ref_mu, ref_X = _eigen_reference(G, F, normY2, delta2)
        mu = torch.tensor(warm, dtype=torch.float64, device="cuda")
        info = torch.full((1,), -7, dtype=torch.int32, device="cuda")
        gen = panel.epc_step64_gen(Gd, Fd, normY2, delta2, mu, info=info)
        try:
            ev = next(gen)
            while True:
                ev.synchronize()
                ev = gen.send(None)
        except StopIteration as stop:
            X = stop.value
        assert int(info) == 0, (delta2, warm)
        got = float(mu)
        if ref_mu == 0.0:
            assert got == 0.0
        else:
            assert abs(got - ref_mu) <= 1e-8 * ref_mu, (delta2, warm, got, ref_mu)
        assert _rel(X, ref_X) < 1e-9, (delta2, warm, _rel(X, ref_X))
        if n <= panel.SPD_SMALL_MAX:
            mu2 = torch.tensor(warm, dtype=torch.float64, device="cuda")
            X2 = panel.epc_step64(Gd, Fd, normY2, delta2, mu2)
            assert _rel(X, X2) < 1e-9


@pytest.mark.parametrize("n", [60, 400])
def test_epc_step_near_singular_gram(n):
    """A rank-deficient, numerically indefinite G (the kind of Hadamard-of-Grams matrix on which
    the library eigensolver failed to converge, round 5), the constraint's root at a shift of
    1e-3 of G's scale: the first evaluations (mu = 0 and below the root) cannot be factorised;
    the device step treats that as a shift too small and returns mu and X within 1e-6 of the
    eigen form, info 0 (one-workgroup form at n = 60, blocked at n = 400). (Far closer to 0,
    e(mu) is flat to fp64 rounding: the search stops at e's rounding floor, where mu is
    ill-determined and only X matters - a CPU emulation of epc_search.h gives the device's mu.)"""
    from admmq import panel
    g = torch.Generator().manual_seed(n + 11)
    B = torch.randn(n, n // 3, generator=g, dtype=torch.float64)
    G = B @ B.T
    G = 0.5 * (G + G.T)
    G[1, 1] -= 1e-9 * float(G.diagonal().mean())
    F = torch.randn(7, n, generator=g, dtype=torch.float64) @ G   # F in G's range (cp_anc's F = Y Z)
    s, V = torch.linalg.eigh(G)
    assert float(s.min()) < 0.0                                   # numerically indefinite
    s = s.clamp_min(0.0)
    Ft = F @ V
    c = torch.sum(Ft * Ft, dim=0)
    mu_t = 1e-3 * float(s.max())
    normY2 = float((F * F).sum())
    delta2 = normY2 - float(torch.sum(c * (s + 2 * mu_t) / (s + mu_t) ** 2))
    ref_mu, ref_X = _eigen_reference(G, F, normY2, delta2)
    mu = torch.zeros((), dtype=torch.float64, device="cuda")
    info = torch.full((1,), -7, dtype=torch.int32, device="cuda")
    X = panel.epc_step64(G.cuda(), F.cuda(), normY2, delta2, mu, info=info)
    assert int(info) == 0
    assert bool(torch.isfinite(X).all())
    assert abs(float(mu) - ref_mu) <= 1e-6 * ref_mu, (float(mu), ref_mu)
    assert _rel(X, ref_X) < 1e-6, _rel(X, ref_X)


@pytest.mark.parametrize("shape,R", [((64, 64, 9), 134), ((128, 64, 9), 183)])
def test_drivers_match_oracle_at_layer_sizes(shape, R):
    """parafac (5 CP-ALS iterations) and cp_anc (5 EPC iterations) on a resnet layer shape
    against the oracle's run of the same algorithm from the same start: weights and factors
    within 1e-6 (R = 134: the one-workgroup solves; R = 183: the blocked ones)."""
    from admmq import parafac_epc as pe
    g = torch.Generator().manual_seed(R)
    Y = torch.randn(*shape, generator=g, dtype=torch.float64) * (2.0 / (shape[0] * 9)) ** 0.5
    w, fs = pe.parafac(Y.cuda(), R, random_state=5, tol=0.0, n_iter_max=5, normalize_factors=True)
    wo, fso = eo.parafac(Y, R, random_state=5, tol=0.0, n_iter_max=5, normalize_factors=True)
    assert _rel(w, wo) < 1e-6, _rel(w, wo)
    for f, fo in zip(fs, fso):
        assert _rel(f, fo) < 1e-6, _rel(f, fo)
    delta = float((Y - eo._reconstruct(wo, fso)).norm())
    w2, fs2 = pe.cp_anc(Y.cuda(), R, delta, wo.cuda(), [f.cuda() for f in fso], maxiter=5, tol=0.0)
    w2o, fs2o = eo.cp_anc(Y, R, delta, wo, fso, maxiter=5, tol=0.0)
    assert _rel(w2, w2o) < 1e-6, _rel(w2, w2o)
    for f, fo in zip(fs2, fs2o):
        assert _rel(f, fo) < 1e-6, _rel(f, fo)
    err = float((Y - eo._reconstruct(w2.cpu(), [f.cpu() for f in fs2])).norm())
    assert err <= delta * (1 + 1e-6)


def test_parafac_epc_many_equals_single():
    """The concurrent model-level initialiser (one HIP stream per layer) gives each layer the
    bits of its own parafac_epc call."""
    from admmq import parafac_epc as pe
    g = torch.Generator().manual_seed(3)
    Ys = [torch.randn(*s, generator=g, dtype=torch.float64).cuda() for s in ((32, 16, 9), (24, 40, 9), (9, 30, 20))]
    ranks = [30, 150, 12]
    kw = dict(als_maxiter=6, epc_maxiter=6, epc_rounds=2)
    many = pe.parafac_epc_many(Ys, ranks, **kw)
    for Y, R, (lm, us) in zip(Ys, ranks, many):
        lm1, us1 = pe.parafac_epc(Y, R, **kw)
        assert torch.equal(lm, lm1)
        for a, b in zip(us, us1):
            assert torch.equal(a, b)


def test_parafac_epc_layer4_timing():
    """init_factors('parafac-epc')'s call (50 ALS + 50 EPC iterations per round, source/admm.py:40-44)
    on resnet18 layer4.0.conv2 (512, 512, 9), R = 1141 - the layer of the reference's published
    parafac-epc numbers (notebooks/Results.ipynb:597-653): no library solve, keeps the ALS error."""
    from admmq import panel, synthetic
    from admmq.parafac_epc import parafac_epc
    idx, spec = synthetic.find_layer("resnet18", "layer4.0.conv2")
    W = torch.from_numpy(synthetic.layer_weight(spec, idx)).cuda().double()
    R = spec.rank()
    assert R == 1141 and R > panel.SPD_SMALL_MAX
    torch.cuda.synchronize()
    t0 = time.time()
    lam, Us = parafac_epc(W, R, als_maxiter=50, epc_maxiter=50, epc_rounds=1)
    torch.cuda.synchronize()
    t = time.time() - t0
    Wc = W.cpu()
    epc_err = float((Wc - eo._reconstruct(lam.cpu(), [u.cpu() for u in Us])).norm() / Wc.norm())
    print(f"parafac-epc layer4.0.conv2 R={R}, one EPC round: {t:.2f} s, rel err {epc_err:.4f}")
    assert all(bool(torch.isfinite(u).all()) for u in Us)
    assert epc_err < 1.0
