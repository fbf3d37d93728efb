"""corr_backward at the train shape for T = 1, 2, 4, 12 lookups (run under rocprofv3 --kernel-trace
to read lookup_bwd_fold_kernel's duration per T: the slope is the per-lookup cost, the intercept
the zero-init + fold + dC write).  coords: 'grid' (regular taps) or 'int' (integer pixel grid,
the cold-start first iteration: irregular tap floors)."""
import sys

import torch

sys.path.insert(0, "e-raft_amd")
from eraft_amd import _lib  # noqa: E402
from eraft_amd.corr import _alloc_grad_pyramid  # noqa: E402

B, D, H, W, L, r = 8, 256, 36, 48, 4, 4
K = (2 * r + 1) ** 2
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(B, D, H, W, device=dev, generator=g)
f2 = torch.randn(B, D, H, W, device=dev, generator=g)
ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                        torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
base = torch.stack([xs, ys])[None].expand(B, 2, H, W)
kind = sys.argv[1] if len(sys.argv) > 1 else "grid"
algo = _lib._ALGOS[sys.argv[2]] if len(sys.argv) > 2 else None
coords = [(base + (0 if kind == "int" else 2.0 * torch.randn(B, 2, H, W, device=dev, generator=g))).contiguous()
          for _ in range(12)]
gouts = [torch.randn(B, L * K, H, W, device=dev, generator=g) for _ in range(12)]
gpyr = _alloc_grad_pyramid(B, H, W, L, f1)
for T in (1, 2, 4, 12):
    for _ in range(5):
        _lib.backward(coords[:T], gouts[:T], r, gpyr, f1, f2, algo)
    torch.cuda.synchronize()
    print("T", T, "done", flush=True)
