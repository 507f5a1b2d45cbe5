"""Factorized-layer export (source/models.py:24-122 layouts): the built layers compute
the convolution / linear map of the reconstructed weight. CPU-only (module construction
is host logic; no HIP kernel involved)."""
import os

import torch
import torch.nn.functional as Fn

from admmq import export


def _rng(seed):
    return torch.Generator().manual_seed(seed)


def test_cp_layer_equals_conv_of_reconstruction():
    g = _rng(0)
    cout, cin, R = 12, 8, 5
    A, B, C = (torch.randn(n, R, generator=g) for n in (cout, cin, 9))
    bias = torch.randn(cout, generator=g)
    W = torch.einsum('ir,jr,kr->ijk', A, B, C).reshape(cout, cin, 3, 3)
    x = torch.randn(2, cin, 11, 11, generator=g)
    for stride, padding in (((1, 1), (1, 1)), ((2, 2), (1, 1)), ((1, 1), (0, 0))):
        seq = export.build_cp_layer(R, [A, B, C], bias, cin, cout, (3, 3), padding, stride, 1)
        ref = Fn.conv2d(x, W, bias, stride=stride, padding=padding)
        torch.testing.assert_close(seq(x), ref, rtol=1e-4, atol=1e-4)
    assert list(dict(seq.named_children())) == ['conv1', 'conv2', 'conv3']


def test_cp2conv_fc_and_svd_layers():
    g = _rng(1)
    cout, cin, R = 10, 7, 4
    A, B = torch.randn(cout, R, generator=g), torch.randn(cin, R, generator=g)
    x = torch.randn(3, cin, 5, 5, generator=g)
    seq = export.build_cp2conv_layer(R, [A, B], None, cin, cout, (0, 0), (2, 2))
    ref = Fn.conv2d(x, (A @ B.T)[:, :, None, None], None, stride=2)
    torch.testing.assert_close(seq(x), ref, rtol=1e-4, atol=1e-4)
    # build_cpfc_layer takes [B, A]: fc1 = A^T (fin -> R), fc2 = B (R -> fout)
    fin, fout = 9, 6
    Bf, Af = torch.randn(fout, R, generator=g), torch.randn(fin, R, generator=g)
    bias = torch.randn(fout, generator=g)
    v = torch.randn(4, fin, generator=g)
    seq = export.build_cpfc_layer(R, [Bf, Af], bias, fin, fout)
    torch.testing.assert_close(seq(v), v @ (Bf @ Af.T).T + bias, rtol=1e-4, atol=1e-4)
    U, Vh = torch.randn(fout, R, generator=g), torch.randn(R, fin, generator=g)
    seq = export.build_svd_layer(R, U, Vh, None, fin, fout)
    torch.testing.assert_close(seq(v), v @ (U @ Vh).T, rtol=1e-4, atol=1e-4)


def test_factor_files_round_trip(tmp_path):
    """The calibrate.py naming reads back what factorize.main writes (weights_only load)."""
    g = _rng(2)
    fs = [torch.randn(n, 3, generator=g) for n in (4, 5, 9)]
    prefix = export.factor_prefix(str(tmp_path), 4, "tensor_mseminmax_symmetric", "admm", 42, "layer1.0.conv1",
                                  "random", 3)
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    for m, f in enumerate(fs):
        torch.save(f, prefix + f"mode_{m}.pt")
    got = export.load_factors(prefix, 3)
    assert all(torch.equal(a, b) for a, b in zip(got, fs))
    conv = torch.nn.Conv2d(5, 4, 3, padding=1, bias=True)
    seq = export.factorized_conv(conv, 3, got)
    assert seq.conv3.bias is not None and tuple(seq.conv2.weight.shape) == (3, 1, 3, 3)
