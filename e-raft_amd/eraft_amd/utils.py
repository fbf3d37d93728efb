"""Caller-side helpers the reference pairs with CorrBlock (model/utils.py:24-27)."""
from __future__ import annotations

import torch


def coords_grid(batch: int, ht: int, wd: int, device=None) -> torch.Tensor:
    """Pixel grid [B, 2, H, W]: channel 0 = x (column index), channel 1 = y (row index)."""
    y, x = torch.meshgrid(torch.arange(ht, device=device), torch.arange(wd, device=device),
                          indexing="ij")
    return torch.stack([x, y], dim=0).float()[None].repeat(batch, 1, 1, 1)
