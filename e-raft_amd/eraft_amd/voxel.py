"""DSEC event representation on the MI355X: drop-in for utils/dsec_utils.py:19-64 VoxelGrid.

    vg = VoxelGrid((bins, height, width), normalize=True)       # loader_dsec.py:219
    grid = vg.convert({"x": x, "y": y, "t": t, "p": p})          # loader_dsec.py:245-257

Events are float32 tensors on an MI355X (x, y rectified pixel coordinates, t normalised to
[0, 1] ascending, p in {0, 1}), as the reference's loader prepares them; the result is the
[bins, height, width] float32 grid, computed by corr_voxel_grid (csrc/corr_voxel.hip).  No
CPU fallback: CPU tensors raise.
"""
from __future__ import annotations

import torch

from . import _lib


class VoxelGrid:
    def __init__(self, input_size: tuple, normalize: bool):
        assert len(input_size) == 3
        self.input_size = tuple(int(v) for v in input_size)
        self.nb_channels = self.input_size[0]
        self.normalize = normalize

    def convert(self, events) -> torch.Tensor:
        ev = [events[k] for k in ("x", "y", "t", "p")]
        dev = ev[0].device
        if dev.type != "cuda":
            raise RuntimeError("VoxelGrid.convert: events must be on an MI355X (HIP) device: "
                               "eraft_amd has no CPU fallback")
        ev = [v.to(dev, torch.float32).contiguous().view(-1) for v in ev]
        out = torch.empty(self.input_size, dtype=torch.float32, device=dev)
        _lib.voxel_grid(*ev, out, self.normalize)
        return out
