"""Event representations on the MI355X.

DSEC: drop-in for utils/dsec_utils.py:19-64 VoxelGrid.

    vg = VoxelGrid((bins, height, width), normalize=True)       # loader_dsec.py:219
    grid = vg.convert({"x": x, "y": y, "t": t, "p": p})          # loader_dsec.py:245-257

Events are float32 tensors on an MI355X (x, y rectified pixel coordinates, t normalised to
[0, 1] ascending, p in {0, 1}), as the reference's loader prepares them; the result is the
[bins, height, width] float32 grid, computed by corr_voxel_grid (csrc/corr_voxel.hip).  No
CPU fallback: CPU tensors raise.

MVSEC: drop-in for utils/transformers.py:18-126 EventSequenceToVoxelGrid_Pytorch.

    voxel = EventSequenceToVoxelGrid(num_bins=5, normalize=True)   # loader_mvsec_flow.py:35
    grid = voxel(event_sequence)   # .features [N, 4] (t, x, y, p), .image_width, .image_height

computed by corr_voxel_grid_tbilinear.  The reference builds on the CPU unless gpu=True; here
the grid is always built on the MI355X (device gpu_nr) and returned there.
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


class EventSequenceToVoxelGrid:
    """utils/transformers.py:18-126: temporal-bilinear voxel grid of an event sequence."""

    def __init__(self, num_bins, gpu=True, gpu_nr=0, normalize=True, forkserver=True):
        # gpu / forkserver are accepted for signature compatibility (transformers.py:20-34):
        # there is no CPU path, and no worker start method is touched here
        assert num_bins > 0
        self.num_bins = int(num_bins)
        self.normalize = normalize
        self.device = torch.device("cuda", gpu_nr)

    def __call__(self, event_sequence) -> torch.Tensor:
        feats = event_sequence.features
        width, height = int(event_sequence.image_width), int(event_sequence.image_height)
        assert feats.shape[1] == 4 and width > 0 and height > 0  # transformers.py:51-54
        ev = torch.as_tensor(feats).to(self.device, torch.float64).contiguous()  # :46, :58-60
        out = torch.empty((self.num_bins, height, width), dtype=torch.float32, device=self.device)
        _lib.voxel_grid_tbilinear(ev, out, self.normalize)
        return out
