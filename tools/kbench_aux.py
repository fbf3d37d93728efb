"""Timing of the ops either side of the CorrBlock path on one MI355X (run via gpurun):
event -> voxel grid (DSEC 15 x 480 x 640, 1M events), warm-start forward splat (60 x 80) and
convex upsampling (60 x 80 -> 480 x 640).  HIP events around 20 back-to-back calls; the C
oracle (sequential CPU restatement, 1 core) timed beside it."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "e-raft_amd"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import prng  # noqa: E402
from eraft_amd import VoxelGrid, _lib, forward_interpolate_pytorch  # noqa: E402
from oracle import oracle  # noqa: E402

dev = "cuda:0"


def gpu_us(fn, rep=20):
    fn()
    torch.cuda.synchronize()
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(rep):
        fn()
    z.record()
    z.synchronize()
    return a.elapsed_time(z) / rep * 1e3


def graph_us(fn, rep=20, trials=5):
    """Per-call time of fn replayed from one HIP graph of rep back-to-back calls (no host overhead)."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(rep):
                fn()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(trials):
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            g.replay()
            z.record(s)
            z.synchronize()
            ts.append(a.elapsed_time(z) / rep * 1e3)
    return sorted(ts)[len(ts) // 2]


def cpu_ms(fn):
    t0 = time.perf_counter()
    fn()
    return (time.perf_counter() - t0) * 1e3


res = {}
M, C, H, W = 1_000_000, 15, 480, 640
u = prng.uniform(71, (4, M))
ev_np = np.stack([(u[0] * W).astype(np.float32), (u[1] * H).astype(np.float32),
                  np.sort(u[2]).astype(np.float32), (u[3] > 0.5).astype(np.float32)])
ev_np[2] = (ev_np[2] - ev_np[2][0]) / (ev_np[2][-1] - ev_np[2][0])
ev = {k: torch.from_numpy(ev_np[i].copy()).to(dev) for i, k in enumerate("xytp")}
vg = VoxelGrid((C, H, W), normalize=True)
res["voxel_grid_dsec_1M_events"] = {"gpu_us": round(gpu_us(lambda: vg.convert(ev)), 1),
                                    "cpu_oracle_ms_1core": round(cpu_ms(lambda: oracle.voxel_grid(ev_np, C, H, W, True)), 1)}
f = prng.gauss(72, (1, 2, 60, 80), 4.0)
ft = torch.from_numpy(f).to(dev)
res["forward_splat_60x80"] = {"gpu_us": round(gpu_us(lambda: forward_interpolate_pytorch(ft)), 1),
                              "cpu_oracle_ms_1core": round(cpu_ms(lambda: oracle.forward_splat(f)), 2)}
mask = torch.randn(1, 576, 60, 80, device=dev)
out = torch.empty(1, 2, 480, 640, device=dev)
res["convex_upsample_60x80"] = {"gpu_us": round(gpu_us(lambda: _lib.convex_upsample(ft, mask, out)), 1),
                                "bytes": int(576 * 4800 * 4 + 2 * 4800 * 4 + 2 * 480 * 640 * 4)}
# lookup fused with convc1 vs lookup + conv2d + relu (DSEC, 12 GRU iterations' worth)
from eraft_amd import CorrBlock  # noqa: E402
import torch.nn.functional as F  # noqa: E402
f1 = torch.randn(1, 256, 60, 80, device=dev)
f2 = torch.randn(1, 256, 60, 80, device=dev)
cb = CorrBlock(f1, f2, 4, 4)
co = (torch.stack(torch.meshgrid(torch.arange(60, device=dev), torch.arange(80, device=dev),
                                 indexing="ij")[::-1]).float()[None] + torch.randn(1, 2, 60, 80, device=dev))
wc = torch.randn(256, 324, 1, 1, device=dev) * 0.05
bc = torch.randn(256, device=dev)
cb.lookup_conv(co, wc, bc)  # packs the weight once (cached per weight version)
res["lookup_convc1_dsec"] = {"timing": "per call, replayed from one HIP graph of 20 calls, median of 5",
                             "fused_us": round(graph_us(lambda: cb.lookup_conv(co, wc, bc)), 2),
                             "unfused_us": round(graph_us(lambda: F.relu(F.conv2d(cb(co), wc, bc))), 2),
                             "lookup_only_us": round(graph_us(lambda: cb(co)), 2)}
fused = cb.lookup_conv(co, wc, bc).double()
ref = F.relu(F.conv2d(cb(co).double(), wc.double(), bc.double()))
res["lookup_convc1_dsec"]["max_abs_err_rel_to_max"] = float((fused - ref).abs().max() / ref.abs().max())
print(json.dumps(res))
