"""Synthetic conv/linear weight tensors with the reference's layer shapes.

The reference factorizes pretrained torchvision / HF weights
(``scripts/factorize.py:116-126``, ``scripts/factorize_lowrank.py:121``); none of
them can be downloaded here, so every workload in this repository uses seeded
synthetic weights of exactly the same shapes.

Shapes are taken as the *intended* reshape of ``scripts/factorize.py:140-147``
(commented out in the reference, restored here): a ``k×k`` conv weight
``(cout, cin, kh, kw)`` becomes ``(cout, cin, kh*kw)`` and a ``1×1`` conv or a
linear weight becomes ``(cout, cin)``.

Layer lists follow ``source/layer_map.py:10-31``; the ranks are
``int(numel / sum(shape) / rate)`` (``scripts/factorize.py:157-158``), which
reproduces the hard-coded tables of ``source/rank_map.py:266-340``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np


@dataclass(frozen=True)
class LayerSpec:
    name: str
    shape: Tuple[int, ...]   # (cout, cin, kh*kw) or (cout, cin)
    fan: int                 # cout * kh * kw (kaiming fan_out) used for the init scale

    def rank(self, rate: float = 2.0) -> int:
        numel = int(np.prod(self.shape))
        return int(numel / sum(self.shape) / rate)


def _conv(name: str, cout: int, cin: int, k: int) -> LayerSpec:
    if k == 1:
        return LayerSpec(name, (cout, cin), cout)
    return LayerSpec(name, (cout, cin, k * k), cout * k * k)


def resnet18_layers() -> List[LayerSpec]:
    """The 16 3×3 convs of ``source/layer_map.py:10-13`` (downsample/conv1/fc off)."""
    out = []
    cin = 64
    for li, cout in enumerate([64, 128, 256, 512], start=1):
        for blk in range(2):
            c_in_first = cin if blk == 0 else cout
            out.append(_conv(f"layer{li}.{blk}.conv1", cout, c_in_first, 3))
            out.append(_conv(f"layer{li}.{blk}.conv2", cout, cout, 3))
        cin = cout
    return out


def resnet50_layers() -> List[LayerSpec]:
    """The 48 bottleneck convs of ``source/layer_map.py:24-31``."""
    blocks = {1: 3, 2: 4, 3: 6, 4: 3}
    width = {1: 64, 2: 128, 3: 256, 4: 512}
    out = []
    cin = 64
    for li in range(1, 5):
        w = width[li]
        for b in range(blocks[li]):
            c_in = cin if b == 0 else 4 * w
            out.append(_conv(f"layer{li}.{b}.conv1", w, c_in, 1))
            out.append(_conv(f"layer{li}.{b}.conv2", w, w, 3))
            out.append(_conv(f"layer{li}.{b}.conv3", 4 * w, w, 1))
        cin = 4 * w
    return out


def llama_layers() -> List[LayerSpec]:
    """One Llama-7B decoder layer (``notebooks/LlamaADMMQuant.ipynb`` cell 8)."""
    d, f = 4096, 11008
    out = [LayerSpec(f"self_attn.{p}_proj", (d, d), d) for p in "qkvo"]
    out += [LayerSpec("mlp.gate_proj", (f, d), f), LayerSpec("mlp.up_proj", (f, d), f),
            LayerSpec("mlp.down_proj", (d, f), d)]
    return out


MODELS = {"resnet18": resnet18_layers, "resnet50": resnet50_layers, "llama7b": llama_layers}


def layer_weight(spec: LayerSpec, index: int, replica: int = 0) -> np.ndarray:
    """Seeded synthetic weight: N(0, 2/fan_out) for convs (torchvision kaiming
    fan_out), N(0, 0.02²) for Llama linears. Seed = 1000 + index + 100*replica."""
    rng = np.random.default_rng(1000 + index + 100 * replica)
    std = 0.02 if spec.name.startswith(("self_attn", "mlp")) else float(np.sqrt(2.0 / spec.fan))
    return (rng.standard_normal(spec.shape) * std).astype(np.float32)


def find_layer(model: str, name: str) -> Tuple[int, LayerSpec]:
    for i, s in enumerate(MODELS[model]()):
        if s.name == name:
            return i, s
    raise ValueError(f"unknown layer {name!r} for model {model!r}")
