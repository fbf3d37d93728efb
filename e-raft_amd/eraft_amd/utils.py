"""Caller-side helpers the reference pairs with CorrBlock (model/utils.py:24-27)."""
from __future__ import annotations

import torch


def coords_grid(batch: int, ht: int, wd: int, device=None) -> torch.Tensor:
    """Pixel grid [B, 2, H, W]: channel 0 = x (column index), channel 1 = y (row index)."""
    y, x = torch.meshgrid(torch.arange(ht, device=device), torch.arange(wd, device=device),
                          indexing="ij")
    return torch.stack([x, y], dim=0).float()[None].repeat(batch, 1, 1, 1)


def forward_interpolate_pytorch(flow_in: torch.Tensor) -> torch.Tensor:
    """Drop-in for utils/image_utils.py:52-83 (the warm-start flow_init of the next pair,
    test.py:209): forward splat of a [B, 2, H, W] (or [2, H, W]) flow on the MI355X
    (corr_forward_splat), bit-identical to the reference on CPU.  Returns [B, 2, H, W]."""
    from . import _lib

    flow = flow_in.detach()
    if flow.dim() < 4:
        flow = flow.unsqueeze(0)
    if flow.device.type != "cuda":
        raise RuntimeError("forward_interpolate_pytorch: flow must be on an MI355X (HIP) device: "
                           "eraft_amd has no CPU fallback")
    flow = flow.float().contiguous()
    out = torch.empty_like(flow)
    _lib.forward_splat(flow, out)
    return out
