"""Per-config GPU tests: BASELINE.json configs C3 (resnet18, all 16 3x3 convs in ONE
batched call), C4 (resnet50, all 48 convs: 16 3-way + 32 2-way, R 16..1141) and C5
(Llama-7B 2-way shapes (4096,4096) R=1024 and (11008,4096) R=1492).

For every problem of a config, one batched ADMM step (both solve forms):
  * H_T within 1e-5 rel-Frobenius of the CPU oracle (scipy float32 Cholesky, the
    reference's formulation; C5: an fp64 solve);
  * the projection bit-exact: the oracle quantizer (oracle/quant_oracle_c.c) applied to
    the kernel's own X = H_T - U equals the kernel's H;
  * the dual update bit-exact: U = U0 + (H - H_T);
and, over 3 inner iterations, the batched call equals per-problem calls bit-for-bit.
Inputs: synthetic weights of the configs' shapes (admmq.synthetic), seed-42 random init,
F/G from the oracle's Gram/MTTKRP (C5: torch matmuls).
"""
import numpy as np
import pytest

from conftest import gpu_available
from oracle import admm_oracle as ao
from oracle import quant_oracle_c as qc

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

MSE = "tensor_mseminmax_symmetric"


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch, torch.device("cuda:0")


def _t(torch, dev, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _config_problems(model, mode):
    """[(name, H0, F, G)] for `mode` of every layer of `model` that has that mode."""
    import torch
    from admmq import synthetic
    out = []
    for l, s in enumerate(synthetic.MODELS[model]()):
        if mode >= len(s.shape):
            continue
        W = synthetic.layer_weight(s, l)
        R = s.rank()
        g = torch.Generator().manual_seed(42)
        fs = [torch.randn(n, R, generator=g).numpy() for n in W.shape]
        G, F = ao.gram_mttkrp(W, fs, mode)
        out.append((s.name, fs[mode], F, G))
    return out


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _check_step(torch, dev, probs, solve, ref_solver):
    from admmq import admm_iteration_batched
    from admmq._lib import solve_mode
    rng = np.random.default_rng(9)
    U0s = [(rng.standard_normal(H.shape) * 1e-3).astype(np.float32) for (_, H, _, _) in probs]
    ps = [(_t(torch, dev, H), _t(torch, dev, U0), _t(torch, dev, F), _t(torch, dev, G))
          for (_, H, F, G), U0 in zip(probs, U0s)]
    with solve_mode(solve):
        Hs, dbg = admm_iteration_batched(ps, 2, 1e-8, 4, MSE, debug_outputs=True)
    worst = 0.0
    for (name, H0, F, G), U0, H, (HT, X), p in zip(probs, U0s, Hs, dbg, ps):
        HT, X, H, U = HT.cpu().numpy(), X.cpu().numpy(), H.cpu().numpy(), p[1].cpu().numpy()
        ref = ref_solver(H0, U0, F, G)
        rel = _rel(HT, ref)
        worst = max(worst, rel)
        assert rel < 1e-5, (name, rel)
        assert np.array_equal(_bits(X), _bits((HT - U0).astype(np.float32))), name
        Hq, _ = qc.quantize_mse(X, 4)
        assert np.array_equal(_bits(H), _bits(Hq)), name
        assert np.array_equal(_bits(U), _bits((U0 + (Hq - HT).astype(np.float32)).astype(np.float32))), name
    return worst


def _oracle_ht(H0, U0, F, G):
    _, _, info = ao.admm_iteration(H0, U0, F, G, 2, 1e-8, 4, MSE, return_info=True)
    return info["HT"]


def _batched_equals_single(torch, dev, probs, iters=4):
    from admmq import admm_iteration_batched
    mk = lambda: [(_t(torch, dev, H), torch.zeros(H.shape, device=dev), _t(torch, dev, F), _t(torch, dev, G))  # noqa
                  for (_, H, F, G) in probs]
    ps = mk()
    Hs = admm_iteration_batched(ps, iters, 0.0, 4, MSE)
    for k, (p, H) in enumerate(zip(ps, Hs)):
        q = mk()[k]
        (H1,) = admm_iteration_batched([q], iters, 0.0, 4, MSE)
        assert np.array_equal(_bits(H.cpu().numpy()), _bits(H1.cpu().numpy())), probs[k][0]
        assert np.array_equal(_bits(p[1].cpu().numpy()), _bits(q[1].cpu().numpy())), probs[k][0]


@pytest.mark.parametrize("solve", ["split", "fp32"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_c3_resnet18_all_layers(torch_dev, mode, solve):
    torch, dev = torch_dev
    probs = _config_problems("resnet18", mode)
    assert len(probs) == 16
    worst = _check_step(torch, dev, probs, solve, _oracle_ht)
    print(f"C3 mode {mode} {solve}: worst H_T rel {worst:.2e}")


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_c3_batched_equals_single(torch_dev, mode):
    torch, dev = torch_dev
    _batched_equals_single(torch, dev, _config_problems("resnet18", mode))


@pytest.mark.parametrize("solve", ["split", "fp32"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_c4_resnet50_all_layers(torch_dev, mode, solve):
    torch, dev = torch_dev
    probs = _config_problems("resnet50", mode)
    assert len(probs) == (48 if mode < 2 else 16)
    worst = _check_step(torch, dev, probs, solve, _oracle_ht)
    print(f"C4 mode {mode} {solve}: {len(probs)} problems, worst H_T rel {worst:.2e}")


def test_c4_batched_equals_single(torch_dev):
    torch, dev = torch_dev
    probs = _config_problems("resnet50", 0)
    _batched_equals_single(torch, dev, probs[::3], iters=3)


def test_c4_fused_three_groups_equals_separate(torch_dev):
    """C4 mode 0 (all 48 resnet50 factors, 5.7 M elements): too many 8 k-element search
    units for one resident round, so the search takes three float4 groups per thread
    (k_mse_hist3<.., 3, true>: U re-read for the finalize) and keeps the finalize fused. Its
    H, U and iteration counts equal those of two groups per thread with the separate
    k_finalize_admm launch, bit for bit, with no internal fault."""
    torch, dev = torch_dev
    from admmq import admm_iteration_batched, _lib
    probs = _config_problems("resnet50", 0)

    def run(nv3, fused):
        ps = [(_t(torch, dev, H), torch.zeros(H.shape, device=dev), _t(torch, dev, F), _t(torch, dev, G))
              for (_, H, F, G) in probs]
        with _lib.fin_nv3(nv3), _lib.fused_finalize(fused):
            Hs, info = admm_iteration_batched(ps, 4, 0.0, 4, MSE, return_info=True)
        return [(H.cpu().numpy(), p[1].cpu().numpy()) for H, p in zip(Hs, ps)], info.cpu().numpy()

    a, ia = run(True, True)
    b, ib = run(False, False)
    assert (ia[:, 3] == 0).all() and (ia[:, 4] == 0).all() and np.array_equal(ia[:, :3], ib[:, :3])
    for (ha, ua), (hb, ub), pr in zip(a, b, probs):
        assert np.array_equal(_bits(ha), _bits(hb)) and np.array_equal(_bits(ua), _bits(ub)), pr[0]
    # the three-group plan without the fused finalize (the fault-repair re-run's form: non-fused
    # k_mse_hist3<.., 3, false> with several units per block + k_finalize_admm), and the
    # exhaustive sweep under the same plan (k_mse_hist<.., 3>): the same bits (advisor r04)
    c, ic = run(True, False)
    with _lib.exhaustive_search(True):
        e, ie = run(True, False)
    for info in (ic, ie):
        assert np.array_equal(info[:, :3], ib[:, :3])
    for (hc, uc), (he, ue), (hb, ub), pr in zip(c, e, b, probs):
        assert np.array_equal(_bits(hc), _bits(hb)) and np.array_equal(_bits(uc), _bits(ub)), pr[0]
        assert np.array_equal(_bits(he), _bits(hb)) and np.array_equal(_bits(ue), _bits(ub)), pr[0]


def _llama_problem(torch, dev, I, J, R, seed):
    """2-way mode 0 of W (I, J): F = W B, G = B^T B (scripts/factorize.py:276-277)."""
    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(I, J, generator=g) * 0.02).to(dev)
    A = torch.randn(I, R, generator=g).to(dev)
    B = torch.randn(J, R, generator=g).to(dev)
    return A, W @ B, B.T @ B


def _fp64_ht(H0, U0, F, G):
    import scipy.linalg as sla
    R = G.shape[0]
    rho = np.float32(np.float32(np.sum(np.diag(G).astype(np.float64))) / np.float32(R))
    A = G.astype(np.float64) + float(rho) * np.eye(R)
    P = F.astype(np.float64) + float(rho) * (H0.astype(np.float64) + U0.astype(np.float64))
    return sla.cho_solve(sla.cho_factor(A, lower=True), P.T).T


@pytest.mark.parametrize("solve", ["split", "fp32"])
@pytest.mark.parametrize("I,J,R", [(4096, 4096, 1024), (11008, 4096, 1492)])
def test_c5_llama_shapes(torch_dev, I, J, R, solve):
    torch, dev = torch_dev
    A, F, G = _llama_problem(torch, dev, I, J, R, seed=I + R)
    probs = [("llama", A.cpu().numpy(), F.cpu().numpy(), G.cpu().numpy())]
    worst = _check_step(torch, dev, probs, solve, _fp64_ht)
    print(f"C5 ({I},{J}) R={R} {solve}: H_T rel vs fp64 {worst:.2e}")


def test_wide_tiles_equal_64x64(torch_dev):
    """The 128x128 tiles (a launch with >= kWideMinTiles 64x64 tiles, e.g. the Llama MLP
    factor; two 32-column sub-tiles per wave) compute each element with the same K order
    and MFMA sequence as the 64x64 tiles: a (512, 1141)
    factor solved beside an (11008, 1492) one (wide tiles) equals the same factor solved
    alone (64x64 tiles) bit for bit, over 3 inner iterations, in both solve forms."""
    torch, dev = torch_dev
    from admmq import admm_iteration_batched
    from admmq._lib import solve_mode
    g = torch.Generator().manual_seed(11)

    def prob(I, R):
        B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
        return (torch.randn(I, R, generator=g) * 0.1, torch.randn(I, R, generator=g), B @ B.T + 0.5 * torch.eye(R))

    small, big = prob(512, 1141), prob(11008, 1492)

    def run(ps):
        args = [(H.to(dev), torch.zeros(H.shape, device=dev), F.to(dev), G.to(dev)) for H, F, G in ps]
        Hs = admm_iteration_batched(args, 4, 0.0, 4, MSE)
        return Hs[0].cpu(), args[0][1].cpu()

    for form in ("split", "fp32"):
        with solve_mode(form):
            h1, u1 = run([small, big])
            h2, u2 = run([small])
        assert torch.equal(h1, h2) and torch.equal(u1, u2), form


def _llama_layer_problems(torch, dev, mode, seed=7):
    """Mode `mode` of all 7 matrices of one Llama-7B decoder layer, as bench.py's C5 step
    batches them (notebooks/LlamaADMMQuant.ipynb cell 8 shapes; R = int(numel / sum(shape) / 2)):
    q/k/v/o (4096, 4096) R=1024, gate/up (11008, 4096) R=1492, down (4096, 11008) R=1492.
    Mode 0: F = W B, G = B^T B; mode 1: F = W^T A, G = A^T A (scripts/factorize.py:276-287)."""
    shapes = [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)]
    g = torch.Generator().manual_seed(seed)
    out = []
    for k, (I, J) in enumerate(shapes):
        R = int(I * J / (I + J) / 2.0)
        W = (torch.randn(I, J, generator=g) * 0.02).to(dev)
        A = torch.randn(I, R, generator=g).to(dev)
        B = torch.randn(J, R, generator=g).to(dev)
        if mode == 0:
            out.append((f"m{k}", A, W @ B, B.T @ B))
        else:
            out.append((f"m{k}", B, W.T @ A, A.T @ A))
    return out


@pytest.mark.parametrize("solve", ["fp32", "split"])
@pytest.mark.parametrize("mode", [0, 1])
def test_c5_llama_full_layer_batch(torch_dev, mode, solve):
    """The whole C5 batched call bench.py times (7 matrices, wide tiles, non-fused search):
    every problem's H_T within 1e-5 of an fp64 solve of the reference's formulation
    (source/admm.py:53-57, on the device in fp64 as the checker), the projection
    bit-exact (C oracle on the kernel's own X) and the dual update bit-exact. Covers the
    (4096, R=1492) factors (down mode 0, gate/up mode 1) too."""
    torch, dev = torch_dev
    from admmq import admm_iteration_batched
    probs = _llama_layer_problems(torch, dev, mode)
    rng = np.random.default_rng(21 + mode)
    U0s = [torch.from_numpy((rng.standard_normal(tuple(H.shape)) * 1e-3).astype(np.float32)).to(dev)
           for (_, H, _, _) in probs]
    ps = [(H, U0.clone(), F, G) for (_, H, F, G), U0 in zip(probs, U0s)]
    Hs, dbg = admm_iteration_batched(ps, 2, 1e-8, 4, MSE, debug_outputs=True, solve=solve)
    worst = 0.0
    for (name, H0, F, G), U0, H, (HT, X), p in zip(probs, U0s, Hs, dbg, ps):
        R = G.shape[0]
        rho = (torch.diagonal(G).sum() / R).double()     # fp32 sum, as source/admm.py:53
        A64 = G.double() + rho * torch.eye(R, device=dev, dtype=torch.float64)
        P64 = F.double() + rho * (H0.double() + U0.double())
        ref = torch.cholesky_solve(P64.T, torch.linalg.cholesky(A64)).T
        rel = float(torch.linalg.norm(HT.double() - ref) / torch.linalg.norm(ref))
        worst = max(worst, rel)
        assert rel < 1e-5, (name, rel)
        X, H, U, HT, U0n = (t.cpu().numpy() for t in (X, H, p[1], HT, U0))
        assert np.array_equal(_bits(X), _bits((HT - U0n).astype(np.float32))), name
        Hq, _ = qc.quantize_mse(X, 4)
        assert np.array_equal(_bits(H), _bits(Hq)), name
        assert np.array_equal(_bits(U), _bits((U0n + (Hq - HT).astype(np.float32)).astype(np.float32))), name
    print(f"C5 full layer mode {mode} {solve}: worst H_T rel vs fp64 {worst:.2e}")


def test_fp32_staging_forms_equal(torch_dev):
    """The fp32 64x64 solve tiles have four staging forms (ADMMQ_GEMM_F32_STAGE /
    admmq_debug_set_gemm_stage: k_gemm's global_load_lds with per-lane addresses, and
    k_gemm_f32b's scalar-offset buffer loads with / without the U prefetch, 3- or 2-deep
    ring). The tile, the wave layout, the K order and the epilogue are the
    same, so every element's MFMA chain is too: H and U equal bit for bit over 3 inner
    iterations, on factors whose launch pads the grid to whole rounds (>256 tiles) and on
    one that fits a single round."""
    torch, dev = torch_dev
    from admmq import admm_iteration_batched, _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(5)

    def prob(I, R):
        B = torch.randn(R, 2 * R, generator=g) / (2 * R) ** 0.5
        return (torch.randn(I, R, generator=g) * 0.1, torch.randn(I, R, generator=g), B @ B.T + 0.5 * torch.eye(R))

    sets = [[prob(512, 1141), prob(256, 574), prob(128, 300)], [prob(200, 131)]]

    def run(ps):
        args = [(H.to(dev), torch.zeros(H.shape, device=dev), F.to(dev), G.to(dev)) for H, F, G in ps]
        Hs = admm_iteration_batched(args, 4, 0.0, 4, MSE)
        return [(h.cpu(), a[1].cpu()) for h, a in zip(Hs, args)]

    try:
        for ps in sets:
            res = []
            for stage in (0, 1, 2, 3):
                _lib.check(lib.admmq_debug_set_gemm_stage(stage), "gemm_stage")
                res.append(run(ps))
            for r in res[1:]:
                for (h0, u0), (h1, u1) in zip(res[0], r):
                    assert torch.equal(h0, h1) and torch.equal(u0, u1)
    finally:
        _lib.check(lib.admmq_debug_set_gemm_stage(3), "gemm_stage")


def test_ksplit_factors(torch_dev):
    """K-split solve tiles (api.hip ksplit_pieces: the pieces are fixed by the factor's
    shape; gemm_kernels.hip: run in parallel by np workgroups with the ksplit_combine
    hand-off, or folded serially by one workgroup - the same float32 sums): the lone
    layer4 conv factor (512, 1141) -> 3 pieces, (512, 759) -> 2, (256, 759) -> 4,
    (256, 566) -> 3. For each: H_T within 1e-5 of the oracle (source/admm.py:56, scipy
    float32 Cholesky) and within 1e-6 of the unsplit solve; the projection bit-exact on
    the kernel's own X; over 4 inner iterations the parallel form (twice: the piece that
    completes a tile varies from run to run, the piece-order sum does not), the serial
    form and the launch's own choice bit-identical."""
    torch, dev = torch_dev
    from admmq import admm_iteration_batched, _lib
    lib = _lib.load()
    expect = {(512, 1141): 3, (512, 759): 2, (256, 759): 4, (256, 566): 3}
    for (I, R), np_ in expect.items():
        assert lib.admmq_debug_ksplit_pieces(I, R) == np_, (I, R)
    rng = np.random.default_rng(3)
    probs = []
    for (I, R) in expect:
        B = rng.standard_normal((R, 2 * R)).astype(np.float32) / np.float32(np.sqrt(2 * R))
        G = (B @ B.T + 0.5 * np.eye(R)).astype(np.float32)
        probs.append((f"{I}x{R}", rng.standard_normal((I, R)).astype(np.float32),
                      rng.standard_normal((I, R)).astype(np.float32), G))
    worst = _check_step(torch, dev, probs, "fp32", _oracle_ht)
    args = lambda: [(_t(torch, dev, H), torch.zeros(H.shape, device=dev), _t(torch, dev, F), _t(torch, dev, G))  # noqa
                    for (_, H, F, G) in probs]

    def run(iters, debug=False):
        ps = args()
        Hs, dbg = admm_iteration_batched(ps, iters, 0.0, 4, MSE, debug_outputs=True)
        return [h.cpu() for h in Hs] + [p[1].cpu() for p in ps], [d[0].cpu() for d in dbg]

    try:
        outs = []
        for form in (2, 2, 0, 1):   # parallel, parallel, serial, launch's choice
            _lib.check(lib.admmq_debug_set_ksplit_form(form), "ksplit_form")
            outs.append(run(4)[0])
        for o in outs[1:]:
            for a, b in zip(outs[0], o):
                assert torch.equal(a, b)
        _lib.check(lib.admmq_debug_set_ksplit_form(1), "ksplit_form")
        _, ht1 = run(2)   # one step, split vs unsplit: the same H_T up to the fp32 summation order
        _lib.check(lib.admmq_debug_set_ksplit(0), "ksplit")
        _, ht0 = run(2)
        for (name, *_), a, b in zip(probs, ht1, ht0):
            assert _rel(a.numpy(), b.numpy()) < 1e-6, name
    finally:
        _lib.check(lib.admmq_debug_set_ksplit(1), "ksplit")
        _lib.check(lib.admmq_debug_set_ksplit_form(1), "ksplit_form")
    print(f"K-split factors: worst H_T rel {worst:.2e}")
