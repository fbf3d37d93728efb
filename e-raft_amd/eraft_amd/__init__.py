"""eraft_amd — MI355X-native E-RAFT correlation hot path (CorrBlock build + lookup + backward).

Product path: Python (this package) -> ctypes -> libcorr_mi355x.so (hand-written gfx950 HIP
kernels behind the C-ABI of include/corr_mi355x.h).  See DESIGN.md.
"""
from .corr import CorrBlock, level_shapes  # noqa: F401
from .utils import coords_grid, forward_interpolate_pytorch  # noqa: F401
from .voxel import EventSequenceToVoxelGrid, VoxelGrid  # noqa: F401

__all__ = ["CorrBlock", "EventSequenceToVoxelGrid", "VoxelGrid", "coords_grid", "forward_interpolate_pytorch", "level_shapes"]
