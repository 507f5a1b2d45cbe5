"""GPU parity of the ALS-sweep contractions (C-ABI admmq_cp_gram_mttkrp / admmq_cp_rel_error):
Gram∘Gram (G1), MTTKRP (M1) and the fused reconstruction error (E1) of
scripts/factorize.py:215-253 / :276-300.

Tolerances (fp32 MFMA products, different summation order than torch's CPU einsum):
  * vs the reference's own G/F fixtures (tests/golden/f2_admm.npz): rel-Frob <= 1e-5;
  * vs a float64 restatement at full resnet18 / Llama shapes: rel-Frob <= 1e-5;
  * error vs the reference's recorded losses (tests/golden/f3_als.npz): rel <= 1e-5;
  * batched == single and reruns: bit-identical (fixed-order split-K and block sums).
"""
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-5


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


def _ref64(torch, W, fs, mode):
    """float64 on the device: G = Hadamard of Grams, F = unfold(W, mode) @ KhatriRao(others)."""
    W = W.double()
    fs = [f.double() for f in fs]
    others = [d for d in range(W.dim()) if d != mode]
    G = torch.ones(fs[0].shape[1], fs[0].shape[1], dtype=torch.float64, device=W.device)
    for d in others:
        G = G * (fs[d].T @ fs[d])
    unf = torch.movedim(W, mode, 0).reshape(W.shape[mode], -1)
    kr = fs[others[0]]
    for d in others[1:]:
        kr = (kr[:, None, :] * fs[d][None, :, :]).reshape(-1, kr.shape[1])
    return G.cpu().numpy(), (unf @ kr).cpu().numpy()


def test_gram_mttkrp_reference_fixtures(torch_dev):
    """G and F of resnet18 layer1.0.conv1 (all 3 modes) and the 2-way case against the
    reference's own torch outputs (F2)."""
    torch, dev = torch_dev
    from admmq.als import gram_mttkrp
    z = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    W = _t(torch, dev, z["l1_W"])
    fs = [_t(torch, dev, z["l1_" + k]) for k in "ABC"]
    for m in range(3):
        G, F = gram_mttkrp(W, fs, m)
        assert _rel(G.cpu().numpy(), z[f"l1_m{m}_G"]) < TOL, m
        assert _rel(F.cpu().numpy(), z[f"l1_m{m}_F"]) < TOL, m
        assert torch.equal(G, G.T), "Gram product must be exactly symmetric"
    W2 = _t(torch, dev, z["w2_W"])
    f2 = [_t(torch, dev, z["w2_A"]), _t(torch, dev, z["w2_B"])]
    G, F = gram_mttkrp(W2, f2, 0)
    assert _rel(G.cpu().numpy(), z["w2_G"]) < TOL
    assert _rel(F.cpu().numpy(), z["w2_F"]) < TOL


@pytest.mark.parametrize("layer", ["layer1.0.conv1", "layer2.0.conv1", "layer3.0.conv2", "layer4.0.conv2"])
def test_gram_mttkrp_resnet_shapes(torch_dev, layer):
    torch, dev = torch_dev
    from admmq import synthetic
    from admmq.als import gram_mttkrp
    idx, spec = synthetic.find_layer("resnet18", layer)
    W = _t(torch, dev, synthetic.layer_weight(spec, idx))
    g = torch.Generator().manual_seed(7)
    fs = [torch.randn(n, spec.rank(), generator=g).to(dev) for n in W.shape]
    for m in range(3):
        G, F = gram_mttkrp(W, fs, m)
        Gr, Fr = _ref64(torch, W, fs, m)
        assert _rel(G.cpu().numpy(), Gr) < TOL, (layer, m)
        assert _rel(F.cpu().numpy(), Fr) < TOL, (layer, m)


@pytest.mark.parametrize("shape,R", [((64, 64), 16), ((256, 64), 25), ((2048, 512), 204), ((11008, 4096), 1492)])
def test_gram_mttkrp_two_way(torch_dev, shape, R):
    """1x1 convs of resnet50 and the Llama-7B MLP shape (scripts/factorize.py:276-287)."""
    torch, dev = torch_dev
    from admmq.als import gram_mttkrp
    g = torch.Generator().manual_seed(3)
    W = (torch.randn(*shape, generator=g) * 0.02).to(dev)
    fs = [torch.randn(n, R, generator=g).to(dev) for n in shape]
    for m in range(2):
        G, F = gram_mttkrp(W, fs, m)
        Gr, Fr = _ref64(torch, W, fs, m)
        assert _rel(G.cpu().numpy(), Gr) < TOL, (shape, m)
        assert _rel(F.cpu().numpy(), Fr) < TOL, (shape, m)


@pytest.mark.parametrize("shape,R", [((48, 40, 9), 20), ((20, 12, 9), 7), ((100, 64, 9), 300), ((96, 64, 25), 30)])
def test_gram_mttkrp_ragged_three_way(torch_dev, shape, R):
    """Ragged 3-way shapes: row tiles past M, R past a 64-column tile, reduction extents
    off the 16-step (the generic Khatri-Rao path) and a 5 x 5 kernel, per mode."""
    torch, dev = torch_dev
    from admmq.als import gram_mttkrp
    g = torch.Generator().manual_seed(13)
    W = (torch.randn(*shape, generator=g) * 0.05).to(dev)
    fs = [torch.randn(n, R, generator=g).to(dev) for n in shape]
    for m in range(3):
        G, F = gram_mttkrp(W, fs, m)
        Gr, Fr = _ref64(torch, W, fs, m)
        assert _rel(G.cpu().numpy(), Gr) < TOL, (shape, m)
        assert _rel(F.cpu().numpy(), Fr) < TOL, (shape, m)


def test_rel_error_reference_fixture(torch_dev):
    """The fused error reproduces the reference's recorded rec / quantized-rec errors
    for the factors it produced (F3: short ALS on layer1.0.conv1 and the 2-way case)."""
    torch, dev = torch_dev
    from admmq.als import rel_error_batched
    z = np.load(os.path.join(GOLDEN, "f3_als.npz"))
    f2 = np.load(os.path.join(GOLDEN, "f2_admm.npz"))
    W = _t(torch, dev, f2["l1_W"])
    W2 = _t(torch, dev, f2["w2_W"])
    fs = [_t(torch, dev, z[f"l1_f{m}"]) for m in range(3)]
    qs = [_t(torch, dev, z[f"l1_q{m}"]) for m in range(3)]
    f2s = [_t(torch, dev, z[f"w2_f{m}"]) for m in range(2)]
    q2s = [_t(torch, dev, z[f"w2_q{m}"]) for m in range(2)]
    e = rel_error_batched([(W, fs), (W, qs), (W2, f2s), (W2, q2s)])
    ref = [z["l1_loss"][-1], z["l1_lossq"][-1], z["w2_loss"][-1], z["w2_lossq"][-1]]
    for got, want in zip(e, ref):
        assert abs(got - want) <= TOL * abs(want), (got, want)


@pytest.mark.parametrize("layer", ["layer1.0.conv1", "layer4.0.conv2"])
def test_rel_error_vs_float64(torch_dev, layer):
    torch, dev = torch_dev
    from admmq import synthetic
    from admmq.als import rel_error
    idx, spec = synthetic.find_layer("resnet18", layer)
    W = _t(torch, dev, synthetic.layer_weight(spec, idx))
    g = torch.Generator().manual_seed(11)
    fs = [(torch.randn(n, spec.rank(), generator=g) * 0.1).to(dev) for n in W.shape]
    rec = torch.einsum('ir,jr,kr->ijk', *[f.double() for f in fs])
    want = float(torch.sqrt(((W.double() - rec) ** 2).sum() / (W.double() ** 2).sum()))
    assert abs(rel_error(W, fs) - want) <= TOL * want


def test_batched_equals_single_and_deterministic(torch_dev):
    torch, dev = torch_dev
    from admmq import synthetic
    from admmq.als import gram_mttkrp, gram_mttkrp_batched, rel_error, rel_error_batched
    layers = []
    g = torch.Generator().manual_seed(5)
    for name in ("layer1.0.conv1", "layer4.0.conv1", "layer2.1.conv2"):
        idx, spec = synthetic.find_layer("resnet18", name)
        W = _t(torch, dev, synthetic.layer_weight(spec, idx))
        layers.append((W, [torch.randn(n, spec.rank(), generator=g).to(dev) for n in W.shape]))
    W2 = (torch.randn(256, 64, generator=g) * 0.05).to(dev)
    layers.append((W2, [torch.randn(n, 25, generator=g).to(dev) for n in W2.shape]))
    for m in range(3):
        sel = [L for L in layers if m < L[0].dim()]
        batch = gram_mttkrp_batched(sel, m)
        again = gram_mttkrp_batched(sel, m)
        for (W, fs), (G, F), (G2, F2) in zip(sel, batch, again):
            Gs, Fs = gram_mttkrp(W, fs, m)
            assert torch.equal(G, Gs) and torch.equal(F, Fs)
            assert torch.equal(G, G2) and torch.equal(F, F2)
    e = rel_error_batched(layers)
    assert e == rel_error_batched(layers)
    assert e == [rel_error(W, fs) for W, fs in layers]


def test_bad_arguments_raise(torch_dev):
    torch, dev = torch_dev
    from admmq.als import gram_mttkrp
    W = torch.zeros(4, 5, 6, device=dev)
    with pytest.raises(ValueError):
        gram_mttkrp(W, [torch.zeros(4, 3, device=dev), torch.zeros(5, 3, device=dev)], 0)
    with pytest.raises(ValueError):
        gram_mttkrp(W, [torch.zeros(4, 3, device=dev), torch.zeros(5, 3, device=dev), torch.zeros(6, 2, device=dev)], 0)
    with pytest.raises(RuntimeError):
        gram_mttkrp(W.cpu(), [torch.zeros(n, 3) for n in (4, 5, 6)], 0)


def test_init_parafac_epc_on_device(torch_dev):
    """init_factors(init='parafac-epc') (source/admm.py:40-44: 50 ALS + 50 EPC iterations)
    runs on the device and hands float32 factors of the layer's shapes to the ADMM driver;
    objective only (parity unpinned: tensorly / musco absent)."""
    torch, dev = torch_dev
    from admmq import init_factors, synthetic
    from admmq.parafac_epc import _reconstruct
    idx, spec = synthetic.find_layer("resnet18", "layer1.0.conv1")
    W = _t(torch, dev, synthetic.layer_weight(spec, idx))
    fs = init_factors(W, spec.rank(), init="parafac-epc", device=dev, seed=42)
    assert [tuple(f.shape) for f in fs] == [(64, spec.rank()), (64, spec.rank()), (9, spec.rank())]
    assert all(f.dtype == torch.float32 and f.device.type == "cuda" for f in fs)
    assert all(bool(torch.isfinite(f).all()) for f in fs)
