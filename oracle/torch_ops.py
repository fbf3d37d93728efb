"""ORACLE — test infrastructure only: the reference op sequence on torch CPU.

The reference CorrBlock never runs on the GPU box (the reference tree does not travel), so
the CPU path timed beside the GPU in bench.py (``cpu_baseline``, kind "port") is this
restatement of its ATen op chain, run on the box's host cores:

  build  (model/corr.py:13-27, 52-60): matmul(F1^T, F2) -> / sqrt(D) -> (L-1) x avg_pool2d(2, 2)
  lookup (model/corr.py:29-50, model/utils.py:7-15): per level, offsets + scale -> normalise
          -> grid_sample(align_corners=True, zeros) -> cat -> permute().contiguous()

tests/test_oracle.py checks it against the reference's golden vectors (bit-identical on the
same torch version).  Only tests/ and bench.py's cpu_baseline leg import it.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def cpu_build(fmap1: torch.Tensor, fmap2: torch.Tensor, num_levels: int = 4):
    B, D, H, W = fmap1.shape
    a = fmap1.reshape(B, D, H * W).transpose(1, 2)
    c = torch.matmul(a, fmap2.reshape(B, D, H * W))
    c = c / torch.sqrt(torch.tensor(D).float())
    level = c.reshape(B * H * W, 1, H, W)
    levels = [level]
    for _ in range(num_levels - 1):
        level = F.avg_pool2d(level, 2, stride=2)
        levels.append(level)
    return levels


def cpu_lookup(levels, coords: torch.Tensor, radius: int = 4) -> torch.Tensor:
    B, _, H, W = coords.shape
    S = 2 * radius + 1
    off = torch.arange(-radius, radius + 1, dtype=torch.float32)
    # component 0 (x) takes the slow window index, component 1 (y) the fast one (corr.py:37-43)
    ox = off.view(S, 1).expand(S, S)
    oy = off.view(1, S).expand(S, S)
    delta = torch.stack([ox, oy], dim=-1).view(1, S, S, 2)
    centre = coords.permute(0, 2, 3, 1).reshape(B * H * W, 1, 1, 2)
    outs = []
    for l, lvl in enumerate(levels):
        h, w = lvl.shape[-2:]
        g = centre / 2 ** l + delta
        gx = 2 * g[..., 0:1] / (w - 1) - 1
        gy = 2 * g[..., 1:2] / (h - 1) - 1
        s = F.grid_sample(lvl, torch.cat([gx, gy], dim=-1), align_corners=True)
        outs.append(s.view(B, H, W, S * S))
    return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous()
