"""Factorized-layer export: CP / low-rank factors -> drop-in ``nn.Sequential`` layers.

Same names, arguments, module layout (``conv1/conv2/conv3``, ``fc1/fc2``, ``vh/u``)
and weight shapes as ``source/models.py:24-122`` (``build_cp_layer``,
``build_cp2conv_layer``, ``build_cpfc_layer``, ``build_svd_layer``), so a model patched
by ``scripts/calibrate.py:150-187`` can take them unchanged. Factors stay on the
device they were produced on (the reference round-trips them through ``.pt`` files):

* 3-way CP of a ``k x k`` conv weight ``W[o, i, h, w] = sum_r A[o,r] B[i,r] C[h k + w, r]``
  becomes 1x1 (B^T) -> depthwise k x k (C) -> 1x1 (A) + bias.
* 2-way CP of a 1x1 conv / linear ``W = A B^T`` becomes two 1x1 convs / linears.

``load_factors`` reads the files ``admmq.factorize.main`` writes, with the
``scripts/calibrate.py:169-184`` naming (``weights_only=True``).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import List, Optional, Sequence, Tuple

import torch
from torch import nn


def _param(t: torch.Tensor) -> nn.Parameter:
    return nn.Parameter(t.detach().clone().contiguous(), requires_grad=True)


def _expect(module_w: torch.Tensor, t: torch.Tensor):
    if tuple(module_w.shape) != tuple(t.shape):
        raise AssertionError(f'Expected shape: {tuple(module_w.shape)}, but got {tuple(t.shape)}')


def build_cp_layer(rank: int, factors: Optional[Sequence[torch.Tensor]], bias: Optional[torch.Tensor], cin: int,
                   cout: int, kernel_size: Tuple[int, int], padding, stride, groups: int = 1) -> nn.Sequential:
    """1x1 (cin -> R) -> depthwise kernel_size (R) -> 1x1 (R -> cout); source/models.py:24-51."""
    dev = factors[0].device if factors else None
    seq = nn.Sequential(OrderedDict([
        ('conv1', nn.Conv2d(cin, rank, kernel_size=(1, 1), groups=groups, bias=False, device=dev)),
        ('conv2', nn.Conv2d(rank, rank, kernel_size=kernel_size, groups=rank, padding=padding, stride=stride,
                            bias=False, device=dev)),
        ('conv3', nn.Conv2d(rank, cout, kernel_size=(1, 1), bias=bias is not None, device=dev)),
    ]))
    if factors:
        A, B, C = factors
        f_cout = A[:, :, None, None]                                        # (cout, R, 1, 1)
        f_cin = B.T[:, :, None, None]                                       # (R, cin, 1, 1)
        f_z = C.reshape(*kernel_size, rank).permute(2, 0, 1)[:, None]       # (R, 1, kh, kw)
        _expect(seq.conv1.weight, f_cin)
        _expect(seq.conv2.weight, f_z)
        _expect(seq.conv3.weight, f_cout)
        with torch.no_grad():
            seq.conv1.weight = _param(f_cin)
            seq.conv2.weight = _param(f_z)
            seq.conv3.weight = _param(f_cout)
            if bias is not None:
                _expect(seq.conv3.bias, bias)
                seq.conv3.bias = _param(bias)
    return seq


def build_cp2conv_layer(rank: int, factors: Optional[Sequence[torch.Tensor]], bias: Optional[torch.Tensor], cin: int,
                        cout: int, padding, stride) -> nn.Sequential:
    """1x1 (cin -> R, with the original padding/stride) -> 1x1 (R -> cout); source/models.py:54-77."""
    dev = factors[0].device if factors else None
    seq = nn.Sequential(OrderedDict([
        ('conv1', nn.Conv2d(cin, rank, kernel_size=(1, 1), padding=padding, stride=stride, bias=False, device=dev)),
        ('conv2', nn.Conv2d(rank, cout, kernel_size=(1, 1), bias=bias is not None, device=dev)),
    ]))
    if factors:
        A, B = factors
        f_cout = A[:, :, None, None]
        f_cin = B.T[:, :, None, None]
        _expect(seq.conv1.weight, f_cin)
        _expect(seq.conv2.weight, f_cout)
        with torch.no_grad():
            seq.conv1.weight = _param(f_cin)
            seq.conv2.weight = _param(f_cout)
            if bias is not None:
                _expect(seq.conv2.bias, bias)
                seq.conv2.bias = _param(bias)
    return seq


def build_cpfc_layer(rank: int, factors: Sequence[torch.Tensor], bias: Optional[torch.Tensor], fin: int,
                     fout: int) -> nn.Sequential:
    """Linear fin -> R (A^T) -> Linear R -> fout (B); source/models.py:80-99 (factors = [B, A])."""
    B, A = factors
    seq = nn.Sequential(OrderedDict([
        ('fc1', nn.Linear(fin, rank, bias=False, device=A.device)),
        ('fc2', nn.Linear(rank, fout, bias=bias is not None, device=A.device)),
    ]))
    _expect(seq.fc1.weight, A.T)
    _expect(seq.fc2.weight, B)
    with torch.no_grad():
        seq.fc1.weight = _param(A.T)
        seq.fc2.weight = _param(B)
        if bias is not None:
            _expect(seq.fc2.bias, bias)
            seq.fc2.bias = _param(bias)
    return seq


def build_svd_layer(rank: int, U: torch.Tensor, Vh: torch.Tensor, bias: Optional[torch.Tensor], fin: int,
                    fout: int) -> nn.Sequential:
    """Linear fin -> R (Vh) -> Linear R -> fout (U); source/models.py:102-122."""
    seq = nn.Sequential(OrderedDict([
        ('vh', nn.Linear(fin, rank, bias=False, device=U.device)),
        ('u', nn.Linear(rank, fout, bias=bias is not None, device=U.device)),
    ]))
    _expect(seq.u.weight, U)
    _expect(seq.vh.weight, Vh)
    with torch.no_grad():
        seq.u.weight = _param(U)
        seq.vh.weight = _param(Vh)
        if bias is not None:
            _expect(seq.u.bias, bias)
            seq.u.bias = _param(bias)
    return seq


def factor_prefix(outdir_root: str, bits: int, qscheme: str, method: str, seed: int, layer: str, init: str,
                  rank: int) -> str:
    """File prefix of scripts/factorize.py:164-166 / scripts/calibrate.py:169-171."""
    return os.path.join(outdir_root, f"{bits}bit_{qscheme}", f"factors_{method}_seed{seed}",
                        f"{layer}_{method}_{init}_rank_{rank}_")


def load_factors(prefix: str, ndim: int, device=None) -> List[torch.Tensor]:
    """``mode_0.pt`` .. ``mode_{ndim-1}.pt`` under ``prefix`` (scripts/calibrate.py:174-181)."""
    out = []
    for m in range(ndim):
        t = torch.load(prefix + f"mode_{m}.pt", map_location="cpu", weights_only=True)
        if t.dtype != torch.float:
            raise TypeError(f"{prefix}mode_{m}.pt: expected float32 factors, got {t.dtype}")
        out.append(t.to(device) if device is not None else t)
    return out


def factorized_conv(conv: nn.Conv2d, rank: int, factors: Sequence[torch.Tensor]) -> nn.Sequential:
    """The replacement scripts/calibrate.py:157-184 builds for ``conv`` from its factors."""
    bias = conv.bias.detach() if conv.bias is not None else None
    if tuple(conv.kernel_size) != (1, 1):
        return build_cp_layer(rank, list(factors), bias, conv.in_channels, conv.out_channels, conv.kernel_size,
                              conv.padding, conv.stride, conv.groups)
    return build_cp2conv_layer(rank, list(factors), bias, conv.in_channels, conv.out_channels, conv.padding,
                               conv.stride)
