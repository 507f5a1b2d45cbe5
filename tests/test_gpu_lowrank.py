"""GPU parity of the quant + low-rank ADMM (admmq.lowrank, C-ABI admmq_lowrank_pre/_post)
against the reference's outputs (tests/golden/f6_lowrank.npz) and the oracle.

  * quantization side: bit-exact (float32 elementwise updates in the reference's order,
    bit-exact quantizer, device break test);
  * rank side (rocSOLVER SVD vs torch-CPU LAPACK): 1e-4 rel-Frobenius (the fixture's
    random 96 x 64 start has close 4th/5th singular values; measured 1.3e-5 after 2 steps);
  * SubspaceProjector vs exact truncation: 1e-4 rel-Frobenius (decaying spectra);
  * KrylovProjector vs exact float64 truncation: 1e-4 on the loop's own flat-spectrum iterates;
  * three outer iterations: rel errors within 1e-3 of the reference's.
"""
import os
from functools import partial

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def env():
    import torch
    return torch, torch.device("cuda:0"), np.load(os.path.join(GOLDEN, "f6_lowrank.npz"))


def _t(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def _rel(a, b):
    return float(np.linalg.norm(np.float64(a) - np.float64(b)) / np.linalg.norm(np.float64(b)))


@pytest.mark.parametrize("qs", ["tensor_minmax", "tensor_mseminmax_symmetric"])
@pytest.mark.parametrize("mi", [2, 3, 50])
def test_quant_side_bit_exact(env, qs, mi):
    torch, dev, z = env
    from admmq import quantize_tensor
    from admmq.lowrank import admm_iteration
    qf = partial(quantize_tensor, qscheme=qs, bits=4)
    H0 = _t(torch, dev, z["Wq0"])
    U = torch.zeros_like(H0)
    H, U2 = admm_iteration(H0, U, _t(torch, dev, z["W"]), _t(torch, dev, z["Wr0"]), qf, rho=1.0, max_iter=mi)
    assert U2 is U                                   # updated in place and returned
    assert torch.equal(H0, _t(torch, dev, z["Wq0"]))   # caller's H untouched
    assert np.array_equal(H.cpu().numpy().view(np.uint32), z[f"{qs}_q_it{mi}_H"].view(np.uint32))
    assert np.array_equal(U.cpu().numpy().view(np.uint32), z[f"{qs}_q_it{mi}_U"].view(np.uint32))


@pytest.mark.parametrize("mi", [2, 3])
def test_rank_side(env, mi):
    torch, dev, z = env
    from admmq.lowrank import admm_iteration, project_rank
    H0 = _t(torch, dev, z["Wr0"])
    H, U = admm_iteration(H0, torch.zeros_like(H0), _t(torch, dev, z["W"]), _t(torch, dev, z["Wq0"]),
                          partial(project_rank, rank=4), rho=1.0, max_iter=mi)
    assert _rel(H.cpu().numpy(), z[f"r_it{mi}_H"]) < 1e-4
    assert _rel(U.cpu().numpy(), z[f"r_it{mi}_U"]) < 1e-4


def test_subspace_projector_matches_svd(env):
    torch, dev, _ = env
    from admmq.lowrank import SubspaceProjector, project_rank
    g = torch.Generator().manual_seed(1)
    for (m, n, r) in ((96, 64, 4), (1024, 768, 16), (4096, 4096, 4)):
        # decaying spectrum (a low-rank-plus-noise weight): the truncation is well defined
        A = (torch.randn(m, r + 8, generator=g) * torch.logspace(0, -1.5, r + 8)) @ torch.randn(r + 8, n, generator=g)
        X = (A + 1e-3 * torch.randn(m, n, generator=g)).to(dev)
        P = SubspaceProjector(r)
        got, want = P(X), project_rank(X, r)
        assert _rel(got.cpu().numpy(), want.cpu().numpy()) < 1e-4, (m, n, r, P.sweeps)
        again = P(X * 1.0001)                       # warm start: converges in a few sweeps
        assert P.sweeps[-1] <= 6, P.sweeps
        assert _rel(again.cpu().numpy(), project_rank(X * 1.0001, r).cpu().numpy()) < 1e-4


def test_krylov_projector_on_the_loops_flat_spectrum_iterate(env):
    """The projection the (f)3 timing uses (KrylovProjector) on the low-rank ADMM's OWN
    inputs at the notebook's shape (q_proj 4096 x 4096, synthetic N(0, 0.02^2), 4-bit
    tensor_minmax, rank 8): their spectrum is flat (sigma_8 / sigma_9 ~ 1 + 1e-3), where a
    subspace iteration stalls. Cold and warm-started, it must agree with the exact float64
    SVD truncation to 1e-4 rel-Frobenius (scripts/factorize_lowrank.py:80-82)."""
    torch, dev, _ = env
    from functools import partial
    from admmq import synthetic
    from admmq.lowrank import KrylovProjector, admm_iteration
    from admmq.quantization import quantize_tensor
    W = torch.from_numpy(synthetic.layer_weight(synthetic.llama_layers()[0], 0)).to(dev)
    g = torch.Generator().manual_seed(42)
    quant = partial(quantize_tensor, qscheme="tensor_minmax", bits=4)
    kry = KrylovProjector(8, seed=42)
    seen = []

    def proj(X):
        seen.append(X.detach().clone())
        return kry(X)
    W_q, U_q = torch.randn(*W.shape, generator=g).to(dev), torch.zeros(W.shape, device=dev)
    W_r = proj(torch.randn(*W.shape, generator=g).to(dev))
    U_r = torch.zeros_like(W_r)
    for _ in range(2):   # two outer iterations of the notebook loop, 4 inner steps each
        W_q, U_q = admm_iteration(W_q, U_q, W, W_r, quant, rho=1.0, max_iter=5)
        W_r, U_r = admm_iteration(W_r, U_r, W, W_q, proj, rho=1.0, max_iter=5)
    for X in (seen[-1], seen[len(seen) // 2]):
        Uu, S, Vt = torch.linalg.svd(X.double(), full_matrices=False)
        exact = (Uu[:, :8] * S[:8]) @ Vt[:8]
        gap = float(S[7] / S[8])
        for P in (KrylovProjector(8, seed=3), kry):   # cold, and warm from the loop's state
            rel = float(torch.linalg.norm(P(X).double() - exact) / torch.linalg.norm(exact))
            print(f"sigma8/sigma9 {gap:.5f}: rel {rel:.2e}, blocks {P.blocks[-1]}")
            assert rel < 1e-4, (gap, rel, P.blocks)


@pytest.mark.parametrize("projection", [None, "svd"])
@pytest.mark.parametrize("qs", ["tensor_minmax", "tensor_mseminmax_symmetric"])
def test_outer_loop_matches_reference(env, qs, projection):
    """The drop-in's default (projection=None: the device Krylov projector on the panel
    kernels) and the explicit exact-SVD projection both follow the reference's F6 outer loop."""
    torch, dev, z = env
    from admmq.lowrank import factorize_lowrank
    kw = {} if projection is None else {"projection": projection}
    Wq, Wr, hist = factorize_lowrank(_t(torch, dev, z["W"]), 4, 4, qs, max_iter=3, seed=42, **kw)
    ref = z[f"{qs}_outer_rel"]
    np.testing.assert_allclose(hist, ref, rtol=1e-3)
    assert _rel(Wr.cpu().numpy(), z[f"{qs}_outer_Wr"]) < 1e-2


def test_device_break_and_large_stream(env):
    torch, dev, _ = env
    from admmq import quantize_tensor
    from admmq.lowrank import admm_iteration
    g = torch.Generator().manual_seed(9)
    W = (torch.randn(4096, 4096, generator=g) * 0.02).to(dev)
    H2 = (torch.randn(4096, 4096, generator=g) * 0.001).to(dev)
    H = torch.randn(4096, 4096, generator=g).to(dev)
    qf = partial(quantize_tensor, qscheme="tensor_minmax", bits=4)
    # one iteration, checked against the same float32 formula evaluated by torch
    U = torch.zeros_like(H)
    Hn, U1, it = admm_iteration(H, U, W, H2, qf, max_iter=2, return_iters=True)
    Hb = (1.0 * (H + 0) + W - H2) / 2.0
    assert it == 1
    assert torch.equal(Hn, qf(Hb - 0))
    assert torch.equal(U1, 0 + (Hn - Hb))
    # eps large: the device test breaks after the first iteration and later ones are no-ops
    _, _, it = admm_iteration(H, torch.zeros_like(H), W, H2, qf, max_iter=40, eps=1e9, return_iters=True)
    assert it == 1


def test_krylov_projector_rank_above_block():
    """KrylovProjector with rank > block (48 > 32): its blocks widen to the rank, so the
    first Rayleigh-Ritz check holds r distinct Ritz pairs (a 32-wide block used to index past
    them and repeat the top singular triplets). Equals the exact float64 truncation
    (scripts/factorize_lowrank.py:80-82) to 1e-6 on a matrix with a decaying spectrum."""
    import torch
    from admmq.lowrank import KrylovProjector
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(4)
    m, n, r = 320, 256, 48
    Uo = torch.linalg.qr(torch.randn(m, n, generator=g, dtype=torch.float64))[0]
    Vo = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))[0]
    s = 0.9 ** torch.arange(n, dtype=torch.float64)
    X = ((Uo * s) @ Vo.T).float()
    Ue, Se, Vte = torch.linalg.svd(X.double(), full_matrices=False)
    exact = (Ue[:, :r] * Se[:r]) @ Vte[:r]
    P = KrylovProjector(r, block=32, seed=1)
    got = P(X.to(dev)).double().cpu()
    assert float(torch.linalg.norm(got - exact) / torch.linalg.norm(exact)) < 1e-6


def test_f10_reference_band():
    """F10 (tests/golden/gen_f10_lowrank.py): the reference's own quant + low-rank loop
    (scripts/factorize_lowrank.py:156-170, inner admm_iteration :85-101) on a 1024 x 1024
    N(0, 0.02^2) weight, 4-bit tensor_minmax, rank 8, 30 outer iterations from its random
    init, plus four reference re-runs from starts ~1 ulp away / at 1 CPU thread. Those
    five runs agree to 2e-4 for 4 outer iterations and then drift apart chaotically (0.28
    by the 30th): the device loop (HIP quantizer + KrylovProjector, the (f)3 timing path)
    from the same seeded start must match the reference's rel_history within 1e-3 for the
    first 4 outer iterations and stay inside the reference's own band (widened by half its
    width + 0.01) for all 30. rel stays above 1 in every reference run: that is the
    reference's behaviour on random-init synthetic weights, not the device loop's."""
    import json
    import torch
    from admmq import quantize_tensor
    from admmq.lowrank import KrylovProjector, admm_iteration
    with open(os.path.join(GOLDEN, "f10_lowrank.json")) as f:
        ref = json.load(f)
    dev = torch.device("cuda:0")
    N, rank, bits = ref["shape"][0], ref["rank"], ref["bits"]
    g = torch.Generator().manual_seed(ref["seed"])
    W = torch.randn(N, N, generator=g) * ref["scale"]
    Wq = torch.randn(N, N, generator=g)
    raw = torch.randn(N, N, generator=g)
    Us, Ss, Vts = torch.linalg.svd(raw)   # the reference's project_rank of its draw (CPU, as it ran)
    Wr = Us[:, :rank] @ torch.diag(Ss[:rank]) @ Vts[:rank]
    W, Wq, Wr = W.to(dev), Wq.to(dev), Wr.to(dev)
    Uq, Ur = torch.zeros_like(Wq), torch.zeros_like(Wr)
    quant = partial(quantize_tensor, qscheme=ref["qscheme"], bits=bits)
    proj = KrylovProjector(rank, seed=0)
    rel = []
    for _ in range(ref["outer"]):
        Wq, Uq = admm_iteration(Wq, Uq, W, Wr, quant, rho=ref["rho"], max_iter=ref["inner_max_iter"])
        Wr, Ur = admm_iteration(Wr, Ur, W, Wq, proj, rho=ref["rho"], max_iter=ref["inner_max_iter"])
        rel.append(float(torch.linalg.norm(W - Wr - Wq) / torch.linalg.norm(W)))
    lo, hi = ref["band_min"], ref["band_max"]
    for i, r in enumerate(rel):
        if i < 4:
            assert abs(r - ref["rel_history"][i]) < 1e-3, (i, r, ref["rel_history"][i])
        w = hi[i] - lo[i]
        assert lo[i] - 0.5 * w - 0.01 <= r <= hi[i] + 0.5 * w + 0.01, (i, r, lo[i], hi[i])
    print("F10 device rel:", [round(r, 4) for r in rel])
