"""Tensor utilities on the hot path (``source/utils.py:60-74``)."""
from __future__ import annotations

import torch


def unfold(tensor: torch.Tensor, mode: int) -> torch.Tensor:
    """Mode-``mode`` unfolding: moveaxis(mode -> 0), reshape (I_mode, -1), row-major."""
    return torch.reshape(torch.moveaxis(tensor, mode, 0), (tensor.shape[mode], -1))
