#!/usr/bin/env python3
"""Benchmark: E-RAFT CorrBlock build + 12 lookups (one frame pair) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Workload (BASELINE.json metric "CorrBlock build+lookup frame-pairs/sec & HBM GB/s at DSEC
480x640"): fmaps [1, 256, 60, 80] fp32 (DSEC 480x640 / 8), 4 levels, radius 4; one step =
CorrBlock(fmap1, fmap2) + 12 lookups at drifting coords (eraft.py:108,127-129) — the whole
hot path, nothing skipped, through the drop-in eraft_amd.CorrBlock (its pyramid and each
lookup's output come from the caching allocator, as in E-RAFT).  Inputs are synthetic and
already resident in HBM.  Each rank processes its own frame pairs (independent units, no
data-path collective) -> weak scaling; value = frame pairs of ALL ranks / max-over-ranks wall
time.

The step is replayed from one HIP graph so the timed loop is not host-launch-bound; after the
W warmup steps, untimed replays continue for 0.25 s (settle()).  Separately, HIP events on the
launch stream bracket graphs of the build alone and of the 12 lookups alone, giving the build
kernels' average durations (-> MFMA roofline) and the per-lookup average (-> HBM roofline).
Rank 0 at N=1 also times the reference op sequence on the host CPU (oracle/torch_ops.py) on
a bounded sample: ``cpu_baseline``.  At N=1 the DSEC line also carries ``workloads``: the same
measurement (value, ms_per_step, roofline, roofline_lookup; train: backward_kernels; train and
mvsec: cpu_baseline) for BASELINE config 4 (train, B8 36x48 forward + backward), config 3
(mvsec, B16 36x44), config 5's 1280x960 and 1920x1280 sizes on one GPU (hires1280, hires1920)
and config 2 (e2e: the full E-RAFT forward, with its CPU baseline), each in the same process.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "e-raft_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "CorrBlock build+lookup frame-pairs/sec & HBM GB/s at DSEC 480×640, 1–8 GPUs"
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E spec
PEAK_F16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense BF16/F16 MFMA
BUILD_ALGO = {0: "fp32", 1: "f16x3", 2: "bf16x6"}
BUILD_KERNELS = {0: "corr_build_kernel", 1: "split_pack_wide_kernel+corr_build_split_kernel",
                 2: "bf16_pack_kernel+corr_build_bf16_kernel"}
PACK_KERNEL = {1: "split_pack_wide_kernel", 2: "bf16_pack_kernel"}
MFMA_KERNEL = {1: "corr_build_split_kernel", 2: "corr_build_bf16_kernel"}
EXEC_FACTOR = {0: 1, 1: 3, 2: 6}  # MFMA products executed per fp32 product
# what "dtype": "f32" means for the build: the arithmetic that forms each fp32 product
BUILD_ARITH = {0: "fp32 MFMA (exact fp32 products, fp32 accumulate; the reference's arithmetic)",
               1: "f16x3 emulated fp32: per-pixel 2^e (hi + lo) f16 split, 3 f16 MFMAs per product "
                  "(hi.hi + hi.lo + lo.hi, ~2^-22 relative: NARROWER than fp32), fp32 accumulate",
               2: "bf16x6, no narrower than fp32: every fp32 feature split EXACTLY into three bf16 pieces "
                  "(hi + mid + lo, fp32's exponent range, no scale or flush), the 6 piece products of "
                  "weight >= 2^-16 on the bf16 MFMA (dropped terms <= 2^-23 |ab|), two fp32 accumulators "
                  "(hi.hi: D/32 roundings per dot product vs D for an fp32 fmaf chain); per-row error vs fp64 "
                  "<= the fp32 MFMA build's (tests/test_gpu_parity.py::test_build_bf16x6_not_narrower_than_fp32)"}
BUILD_NOTE = {
    0: "fp32 operands on v_mfma_f32_32x32x2_f32: achieved = 2*B*N^2*D flops / build kernel time, "
       "against the fp32 MFMA peak",
    1: "fp32 product emulated on the f16 MFMA pipe (per-pixel 2^e*(hi+lo) split, 3 f16 MFMAs per "
       "fp32 product, fp32 accumulate): achieved = EXECUTED f16 flops (3 * 2*B*N^2*D) / (pack + "
       "MFMA kernel time, each kernel timed alone: kernel_us), against the dense f16 MFMA peak; "
       "the fp32-equivalent rate is fp32_equivalent_tflops",
    2: "fp32 product on the bf16 MFMA pipe (exact three-piece bf16 split, 6 bf16 MFMAs per fp32 "
       "product, fp32 accumulate): achieved = EXECUTED bf16 flops (6 * 2*B*N^2*D) / (pack + MFMA "
       "kernel time, each kernel timed alone: kernel_us), against the dense bf16 MFMA peak; the "
       "fp32-equivalent rate (2*B*N^2*D / time) is fp32_equivalent_tflops",
}
# The backward GEMMs' arithmetic per backward algorithm (corr_bwd_split.hip / corr_bwd.hip).
BWD_ARITH = {0: "fp32 operands on the fp32 MFMA",
             1: "f16x3: per-row 2^e (hi + lo) f16 split, 3 f16 MFMAs per product (~2^-22 relative: NARROWER "
                "than fp32)",
             2: "bf16x6: both operands split EXACTLY into three bf16 pieces while staging (no scales), the 6 "
                "piece products of weight >= 2^-16 on the bf16 MFMA into one fp32 accumulator (6 roundings "
                "per 16 k vs 16 for an fp32 fmaf chain): a tighter a-priori bound and smaller worst / mean "
                "row error than the fp32-operand GEMMs, not every single row "
                "(tests/test_gpu_parity.py::test_build_bwd_bf16x6_not_narrower_than_fp32)"}

WORKLOADS = {
    # name: (B, D, H, W, levels, radius, iters)
    "dsec": (1, 256, 60, 80, 4, 4, 12),
    "mvsec": (16, 256, 36, 44, 4, 4, 12),        # config 3, 260x346 padded to 288x352
    "mvsec_crop": (16, 256, 32, 32, 4, 4, 12),   # config 3, the eval's 256x256 centre crop
    "hires1280": (1, 256, 120, 160, 4, 4, 12),   # 1280x960: the 1.47 GB volume
    "hires1920": (1, 256, 160, 240, 4, 4, 12),   # config 5: 1920x1280, 5.9 GB volume
    # BASELINE config 4: training step, batch 8 at 288x384 crops -> CorrBlock forward AND
    # backward (grad w.r.t. both fmaps through all 12 lookups)
    "train": (8, 256, 36, 48, 4, 4, 12),
}
CPU_SKIP = {"hires1280", "hires1920"}  # a CPU pair takes tens of seconds and >10 GB
TRAIN_WORKLOADS = {"train"}
# The default (DSEC) line also measures these BASELINE configs, one `workloads` entry each
# (config 4 train, config 3 MVSEC B16, config 5's 1280x960 and 1920x1280 sizes on one GPU, config 2
# the full E-RAFT forward),
# so the driver's own run times them; --no-workloads skips them.
EXTRA_WORKLOADS = ("train", "mvsec", "hires1280", "hires1920", "e2e")
ACHIEVABLE_HBM_GBS = 6290.0  # MI355X_MICROARCH.md: measured achievable HBM read bandwidth
# The lookup's measured latency floor per workload: the same launch with neither the window
# loads nor the output stores (coords load, taps, barriers, graph launch), i.e. what no change of
# memory traffic can remove (tools/kbench_lookup.hip "abl QB32 noload nostore",
# profiles/r05t_kbench_lookup_ablations.txt; 1920x1280: profiles/r06za_kbench_lookup_1920.txt; median us).
LOOKUP_NOLOAD_NOSTORE_US = {"dsec": 4.19, "mvsec": 11.49, "train": 6.86, "hires1280": 8.54, "hires1920": 14.78}
LOOKUP_FLOOR_SOURCE = {"hires1920": "profiles/r06za_kbench_lookup_1920.txt"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="dsec", choices=sorted(WORKLOADS) + ["e2e"],
                    help="e2e: BASELINE config 2, the full E-RAFT forward (eraft_amd.model) at DSEC "
                         "480x640, warm start, 12 GRU iterations, random-init weights")
    ap.add_argument("--eager", action="store_true", help="launch eagerly instead of HIP graphs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sharded", action="store_true",
                    help="row-shard ONE frame pair's query rows over the ranks (SURVEY §8e): RCCL "
                         "broadcast of fmap2 in target-row chunks, each chunk's build starting on its "
                         "arrival + slab lookups; strong scaling")
    ap.add_argument("--chunks", type=int, default=4, help="--sharded: fmap2 broadcast chunks")
    ap.add_argument("--prefetch", action="store_true",
                    help="--sharded: instead of chunks, double-buffer whole fmap2s across pairs "
                         "(pair k+1's broadcast during pair k; eager)")
    ap.add_argument("--no-sharded-leg", action="store_true",
                    help="N > 1 dsec: skip the row-sharded 1280x960 leg reported beside the replica value")
    ap.add_argument("--no-workloads", action="store_true",
                    help="N = 1 dsec: skip the train / mvsec / hires1280 / hires1920 / e2e entries of `workloads`")
    return ap.parse_args()


def build_flops(B, D, H, W):
    N = H * W
    return 2.0 * B * N * N * D


def build_bytes(B, D, H, W, L):
    N = H * W
    lv = sum((H >> l) * (W >> l) for l in range(L))
    return 2.0 * B * D * N * 4 + B * N * lv * 4


def lookup_bytes(B, H, W, L, r):
    # per query L*(2r+2)^2 read footprint + L*(2r+1)^2 written + 8 B coords
    N = H * W
    return B * N * (L * (2 * r + 2) ** 2 * 4 + L * (2 * r + 1) ** 2 * 4 + 8)


# FETCH_SIZE correction per kernel, calibrated on known byte counts (tools/kbench_fetchcal.hip):
# coalesced streams (16-B or 4-B per lane, and the build's LDS-DMA) report half their bytes (x2, as
# MI355X_MICROARCH.md §HBM states for 16-B streams; profiles/r02ag_fetch_size_calibration.txt), and
# so does the round-5 lookup's tiled window gather (16-B tile-row chunks: half of the 128-B lines
# it touches, profiles/r05m_fetch_size_calibration.txt).  Only rounds 1-4's row-major gather of
# scattered 44-B row segments was counted at face value in 64-B sectors (x1); no profile of that
# layout is read any more (traffic() takes the newest).
FETCH_FACTOR = {}


def traffic(workload, kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (profiles/*_pmc.json,
    written by tools/pmc_summary.py --json): FETCH_SIZE x FETCH_FACTOR (2 unless calibrated
    otherwise) + WRITE_SIZE, in bytes.  The PMC passes are separate rocprofv3 runs of this
    script; null when no profile exists."""
    import glob
    import re

    def tag_order(path):  # r02u < r02z < r02aa < r02ac < r03a: round, then suffix length, then suffix
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}_pmc.json")), key=tag_order)
    if not files:
        return None
    with open(files[-1]) as fh:
        d = json.load(fh)
    k = d.get("kernels", {}).get(kernel)
    if not k or "FETCH_SIZE" not in k or "WRITE_SIZE" not in k:
        return None
    return int(round((FETCH_FACTOR.get(kernel, 2) * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024))


def build_traffic(workload, algo):
    ks = BUILD_KERNELS[algo].split("+")
    t = [traffic(workload, k) for k in ks]
    return None if any(x is None for x in t) else sum(t)


def cpu_baseline(workload, budget_s, train=False, threads=None):
    """The reference op chain on torch CPU, bounded sample.  threads: None = the job's host
    cores (OMP_NUM_THREADS share), 1 = the reference eval's own setting (main.py:2-5).
    train: plus the autograd backward to both fmaps through the 12 lookups (randn grads)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle import torch_ops

    B, D, H, W, L, r, iters = workload
    # the GPU box exposes every host CPU but grants this job a share (OMP_NUM_THREADS)
    cores = threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    g = torch.Generator().manual_seed(0)
    f1 = torch.randn(B, D, H, W, generator=g)
    f2 = torch.randn(B, D, H, W, generator=g)
    base = torch.stack(torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")[::-1]).float()
    coords = [(base[None] + 0.5 * t * torch.randn(B, 2, H, W, generator=g)) for t in range(iters)]

    gouts = [torch.randn(B, L * (2 * r + 1) ** 2, H, W, generator=g) for _ in range(iters)] if train else None
    if train:
        f1.requires_grad_(True)
        f2.requires_grad_(True)

    def pair():
        with torch.set_grad_enabled(train):
            lv = torch_ops.cpu_build(f1, f2, L)
            outs = [torch_ops.cpu_lookup(lv, c, r) for c in coords]
            if train:
                torch.autograd.backward(outs, gouts)
                f1.grad = f2.grad = None

    pair()  # warm
    times = []
    t_end = time.perf_counter() + budget_s
    while (time.perf_counter() < t_end and len(times) < 200) or len(times) < 2:
        t0 = time.perf_counter()
        pair()
        times.append(time.perf_counter() - t0)
    torch.set_num_threads(prev)
    times.sort()
    med = times[len(times) // 2]
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(B / med, 3), "unit": "frame-pairs/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} frame pairs (build + {iters} lookups{' + autograd backward' if train else ''}"
                      f", torch CPU op chain of "
                      f"model/corr.py), median {med * 1e3:.1f} ms, best {times[0] * 1e3:.1f} ms; "
                      f"{cpu}"}


def run_e2e(args, world, rank, dev, role="primary"):
    """BASELINE config 2: full E-RAFT forward (encoders on MIOpen, the HIP CorrBlock, 12 GRU
    iterations, convex upsampling) on 15-bin voxel pairs at 480x640, warm start (flow_init at
    1/8 resolution), random-init weights.  One step = one frame pair, replayed from one HIP
    graph (--eager: launched op by op).  role "workload": return the result (an entry of the
    DSEC line's `workloads`, CPU baseline on half the budget) instead of printing it."""
    from eraft_amd.model import ERAFT
    torch.manual_seed(0)
    bins, H, W, iters = 15, 480, 640, 12
    model = ERAFT({"subtype": "warm_start"}, n_first_channels=bins).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(7 + rank)

    def voxels():
        v = torch.randn(1, bins, H, W, device=dev, generator=g)
        return v * (torch.rand(1, bins, H, W, device=dev, generator=g) < 0.15)

    im1, im2 = voxels(), voxels()
    finit = 2.0 * torch.randn(1, 2, H // 8, W // 8, device=dev, generator=g)
    launch = "eager"
    with torch.no_grad():
        for _ in range(args.warmup):
            model(im1, im2, iters=iters, flow_init=finit)
        torch.cuda.synchronize()
        step = lambda: model(im1, im2, iters=iters, flow_init=finit)  # noqa: E731
        if not args.eager:
            # the whole forward (MIOpen convs, GRU elementwise ops, the HIP CorrBlock) as ONE
            # HIP graph: the GRU loop is otherwise bound by ~70 launches per iteration
            try:
                s = torch.cuda.Stream(device=dev)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    step()
                torch.cuda.current_stream().wait_stream(s)
                gph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gph):
                    step()
                gph.replay()
                torch.cuda.synchronize()
                step, launch = gph.replay, "hipgraph"
            except Exception as exc:  # noqa: BLE001 — report and stay eager
                print(f"e2e: graph capture failed ({exc}); eager", file=sys.stderr)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = {
        "metric": METRIC + " [config 2: full E-RAFT forward]",
        "value": round(args.steps * world / elapsed, 2), "unit": "frame-pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic 15-bin voxel grids (15% nonzero, randn), random-init weights",
        "config": {"workload": "E-RAFT forward, DSEC 480x640 warm start, 12 GRU iters, HIP CorrBlock",
                   "global_batch": world, "launch": launch,
                   "parallelism": f"replicas x{world}"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        budget = args.cpu_seconds * (0.5 if role == "workload" else 1.0)
        res["cpu_baseline"] = cpu_e2e(model, im1, im2, finit, iters, budget)
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
    if role == "workload":
        return res
    if rank == 0:
        emit(res)


def cpu_e2e(model, im1, im2, finit, iters, budget_s):
    """The same model on the host cores with the reference CorrBlock op chain (the oracle's
    torch-CPU restatement of model/corr.py) in place of the HIP one."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle import torch_ops
    import eraft_amd.model as M

    class CpuCorrBlock:
        def __init__(self, f1, f2, num_levels=4, radius=4):
            self.levels, self.radius = torch_ops.cpu_build(f1, f2, num_levels), radius

        def __call__(self, coords):
            return torch_ops.cpu_lookup(self.levels, coords, self.radius)

    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    orig = M.CorrBlock
    M.CorrBlock = CpuCorrBlock
    cpu_model = model.to("cpu")
    a, b, f = im1.cpu(), im2.cpu(), finit.cpu()
    times = []
    try:
        with torch.no_grad():
            cpu_model(a, b, iters=iters, flow_init=f)  # warm
            t_end = time.perf_counter() + budget_s
            while time.perf_counter() < t_end or len(times) < 2:
                t0 = time.perf_counter()
                cpu_model(a, b, iters=iters, flow_init=f)
                times.append(time.perf_counter() - t0)
    finally:
        M.CorrBlock = orig
        torch.set_num_threads(prev)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(1.0 / med, 3), "unit": "frame-pairs/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} full E-RAFT forwards on torch CPU (reference CorrBlock op chain), "
                      f"median {med * 1e3:.0f} ms"}


def settle(step, seconds=0.25, cap=5000, fixed=None):
    """Untimed replays after the W warmup steps until `seconds` have passed: the first ~100 ms of
    replays after a graph capture run 4-5 % slower (clock ramp / first touches of the graph
    pool), which a 10-step warmup at DSEC (1.5 ms) does not cover (tools/ab_api_vs_direct.py).
    fixed = n: exactly n replays instead — a step with collectives (the row-sharded pair) must run
    the same number of times on every rank, which a per-rank clock does not guarantee."""
    if fixed is not None:
        for _ in range(fixed):
            step()
        torch.cuda.synchronize()
        return
    t0 = time.perf_counter()
    n = 0
    while n < cap and time.perf_counter() - t0 < seconds:
        for _ in range(8):
            step()
        n += 8
        torch.cuda.synchronize()


def graph_time_ms(fn, stream, rep=10, trials=5):
    """Median time of one call of fn: REP back-to-back calls captured in one HIP graph,
    bracketed by HIP events on the launch stream (the graph-launch gap is amortised, so the
    per-call figure is the kernels' own duration and agrees with rocprofv3's kernel trace)."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(rep):
            fn()
    times = []
    for _ in range(trials):
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        g.replay()
        z.record(stream)
        z.synchronize()
        times.append(a.elapsed_time(z))
    times.sort()
    return times[len(times) // 2] / rep


def build_roofline(algo, fl, bb, t_ms, traffic_b):
    """The build kernel against the roofline of the pipe it runs on (see BUILD_NOTE)."""
    executed = EXEC_FACTOR[algo] * fl
    peak = PEAK_F16_MFMA_TFLOPS if algo != 0 else PEAK_FP32_MFMA_TFLOPS
    ach = executed / (t_ms * 1e-3) / 1e12
    # The build is bounded by BOTH its pipe and its HBM bytes (the pyramid write); report which
    # floor binds and the fraction of that floor achieved, beside the pipe fraction above.
    t_pipe_us = executed / (peak * 1e12) * 1e6
    t_hbm_us = bb / (PEAK_HBM_GBS * 1e9) * 1e6
    floor_us = max(t_pipe_us, t_hbm_us)
    return {"bound": "mfma", "kernel": BUILD_KERNELS[algo], "achieved": round(ach, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic_b,
            "avg_us": round(t_ms * 1e3, 2), "flops_per_launch": executed, "algorithmic_fp32_flops": fl,
            "fp32_equivalent_tflops": round(fl / (t_ms * 1e-3) / 1e12, 2), "bytes_per_launch": bb,
            "binding_floor": {"bound": "hbm" if t_hbm_us > t_pipe_us else "mfma", "pipe_floor_us": round(t_pipe_us, 2),
                              "hbm_floor_us": round(t_hbm_us, 2), "frac": round(floor_us / (t_ms * 1e3), 4)},
            "note": BUILD_NOTE[algo]}


def lookup_ceiling(wl_name, lb, look_ms, traffic_b):
    """What bounds the lookup short of 8 TB/s, stated as ceilings on `frac`:
    latency_floor — the launch without window loads or output stores (measured, see
    LOOKUP_NOLOAD_NOSTORE_US): algorithmic bytes / that time is the best the kernel's fixed
    chain allows; line_granularity — the window gather moves whole 128-B lines, so the counted
    HBM traffic per launch (PMC) exceeds the algorithmic bytes: at the achievable 6.29 TB/s the
    algorithmic rate is at most (algorithmic / counted) x 6.29 TB/s.  `binding` is the lower."""
    out = {}
    fl = LOOKUP_NOLOAD_NOSTORE_US.get(wl_name)
    if fl:
        gbs = lb / (fl * 1e-6) / 1e9
        out["latency_floor"] = {"noload_nostore_us": fl, "frac": round(gbs / PEAK_HBM_GBS, 4),
                                "source": LOOKUP_FLOOR_SOURCE.get(wl_name, "profiles/r05t_kbench_lookup_ablations.txt")}
    if traffic_b:
        r = min(1.0, lb / traffic_b)
        out["line_granularity"] = {"algorithmic_over_counted": round(r, 4),
                                   "frac": round(r * ACHIEVABLE_HBM_GBS / PEAK_HBM_GBS, 4)}
    if out:
        name, c = min(out.items(), key=lambda kv: kv[1]["frac"])
        frac = lb / (look_ms * 1e-3) / 1e9 / PEAK_HBM_GBS
        out["binding"] = name
        out["frac_of_ceiling"] = round(frac / c["frac"], 4)
    return out


_JSON_OUT = None  # where the one JSON line goes (the process's stdout, see main)


def emit(res):
    """Print the result line (rank 0) on the original stdout."""
    out = _JSON_OUT or sys.stdout
    out.write(json.dumps(res) + "\n")
    out.flush()


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N ranks of this script as child processes (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1), before
    this process touches the GPU, and exit with the first failing rank's status.  Rank 0 prints
    the one JSON line.  Equivalent to `python -m torch.distributed.run --nproc-per-node N`."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for i in range(n):
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:  # a rank failed: the others would wait at a collective forever
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc if rc >= 0 else 128 - rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    if os.environ.get("ERAFT_AMD_DIST_BACKEND", "nccl") != "nccl":  # rehearsal: ranks may share a GPU
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # stdout carries only the JSON line: native libraries' chatter on fd 1 (gloo prints its
        # connection lines there) goes to stderr, the line to the saved original stdout
        global _JSON_OUT
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # nccl = RCCL over xGMI; ERAFT_AMD_DIST_BACKEND=gloo rehearses the multi-rank path with
        # several ranks on ONE GPU (RCCL refuses two ranks per device)
        backend = os.environ.get("ERAFT_AMD_DIST_BACKEND", "nccl")
        # a mismatched collective fails after 5 minutes instead of holding the node for the default 10
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(minutes=5),
                                **({"device_id": dev} if backend == "nccl" else {}))

    if args.workload == "e2e":
        run_e2e(args, world, rank, dev)
    else:
        res = run_corr(args, args.workload, args.sharded, world, rank, dev)
        if world == 1 and not args.sharded and args.workload == "dsec" and not args.no_workloads:
            # BASELINE configs 2, 3, 4 and 5 measured in the same (driver) run, beside `value`
            res["workloads"] = {}
            for wl in EXTRA_WORKLOADS:
                torch.cuda.empty_cache()
                t_w = time.perf_counter()
                try:
                    ent = (run_e2e(args, world, rank, dev, role="workload") if wl == "e2e" else
                           run_corr(args, wl, False, world, rank, dev, role="workload"))
                    same = ("metric", "unit", "higher_is_better") if wl != "e2e" else ()
                    for k in same + ("n_gpus", "vs_baseline", "data", "dtype",
                                     "scaling", "build_arith", "kernel_timing", "warmup"):
                        ent.pop(k, None)
                except Exception as exc:  # noqa: BLE001 — the DSEC line stands; say why the entry is missing
                    ent = {"error": f"{type(exc).__name__}: {exc}"}
                ent["wall_s"] = round(time.perf_counter() - t_w, 2)
                res["workloads"][wl] = ent
        if world > 1 and not args.sharded and args.workload == "dsec" and not args.no_sharded_leg:
            # the north_star's scaling case beside the replica value: ONE 1280x960 pair row-sharded
            # over the N ranks (chunked RCCL broadcast of fmap2, graph-captured), strong scaling
            try:
                leg = run_corr(args, "hires1280", True, world, rank, dev, role="leg")
            except Exception as exc:  # noqa: BLE001 — the replica line above stands; say why the leg is missing
                leg = {"error": f"{type(exc).__name__}: {exc}"}
            if rank == 0:
                res["sharded_hires1280"] = leg
        if rank == 0:
            emit(res)
    if world > 1:
        dist.destroy_process_group()


def run_corr(args, wl_name, sharded, world, rank, dev, role="primary"):
    """One CorrBlock workload: returns the result dict on rank 0 (None elsewhere).  role "leg"
    (the sharded leg of an N > 1 run): no alternative builds, no CPU baseline; "workload" (an
    entry of the DSEC line's `workloads`): no alternative builds, CPU baselines on half the
    sample budget."""
    primary = role == "primary"
    from eraft_amd import CorrBlock, _lib
    from eraft_amd.corr import _alloc_grad_pyramid, _alloc_pyramid

    _lib.load()
    wl = WORKLOADS[wl_name]
    B, D, H, W, L, r, iters = wl
    K = (2 * r + 1) ** 2
    train = wl_name in TRAIN_WORKLOADS
    if sharded and train:
        raise SystemExit("--sharded times the forward path (build + lookups)")
    # sharded: every rank draws the same pair (same seed); rank 0's fmap2 is what the broadcast
    # carries.  replicas: each rank its own pair.
    g = torch.Generator(device=dev).manual_seed(1234 if sharded else 1234 + rank)
    f1 = torch.randn(B, D, H, W, device=dev, generator=g)
    f2 = torch.randn(B, D, H, W, device=dev, generator=g)
    base = torch.stack(torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev),
                                      indexing="ij")[::-1]).float()[None].repeat(B, 1, 1, 1)
    coords = [(base + 0.5 * t * torch.randn(B, 2, H, W, device=dev, generator=g)).contiguous()
              for t in range(iters)]

    if sharded:
        from eraft_amd.sharded import _alloc_pyramid_rows, row_partition
        h0, h1 = row_partition(H, world, rank)
        f1 = f1[:, :, h0:h1].contiguous()
        coords = [c[:, :, h0:h1].contiguous() for c in coords]
        pyr = _alloc_pyramid_rows(B, (h1 - h0) * W, H, W, L, f2)
        outs = [torch.empty(B, L * K, h1 - h0, W, device=dev) for _ in range(iters)]
    else:
        pyr = _alloc_pyramid(B, H, W, L, f1)
        outs = [torch.empty(B, L * K, H, W, device=dev) for _ in range(iters)]

    algo = _lib.default_algo()
    ws = _lib.build_workspace(f1, f2, algo)  # the split operands (BF16X6 / F16X3), reused every step
    ws_x3 = _lib.build_workspace(f1, f2, _lib.BUILD_F16X3)

    def build_only():
        _lib.build(f1, f2, pyr, algo, ws)

    def build_fp32():
        _lib.build(f1, f2, pyr, _lib.BUILD_FP32, None)

    def build_f16x3():
        _lib.build(f1, f2, pyr, _lib.BUILD_F16X3, ws_x3)

    def build_pack():  # the split build's two kernels timed apart (corr_build_ex measurement flags)
        _lib.build(f1, f2, pyr, algo | _lib.BUILD_ONLY_PACK, ws)

    def build_mfma():
        _lib.build(f1, f2, pyr, algo | _lib.BUILD_ONLY_MFMA, ws)

    def run_lookups():  # kernel timing: 12 distinct output buffers (no reuse through the MALL)
        for c, o in zip(coords, outs):
            _lib.lookup(pyr, c, r, o, H, W)

    def run_lookups_reused():  # the step: one output buffer, as the model's caching allocator
        for c in coords:       # hands the freed previous iteration's output to the next lookup
            _lib.lookup(pyr, c, r, outs[0], H, W)

    def api_pair():  # the drop-in CorrBlock: ctor (pyramid + workspace) and 12 __call__s
        cb = CorrBlock(f1, f2, num_levels=L, radius=r)
        for c in coords:
            cb(c)

    if train:
        # backward of the 12 lookups + pyramid + product (eraft.py:128 detaches coords)
        gouts = [torch.randn(B, L * K, H, W, device=dev, generator=g) for _ in range(iters)]
        gpyr = _alloc_grad_pyramid(B, H, W, L, f1, zero=True)
        gbuf = gpyr[0]._base  # the one allocation behind every level view
        f1g = f1.clone().requires_grad_(True)
        f2g = f2.clone().requires_grad_(True)

        def run_bwd_kernels():  # corr_backward alone: all lookup backwards + fold + GEMMs
            return _lib.backward(coords, gouts, r, gpyr, f1, f2)

        def run_bwd_f16x3():  # the same with the narrower f16x3 split GEMMs (+ the maxima they need)
            return _lib.backward(coords, gouts, r, gpyr, f1, f2, _lib.BUILD_F16X3)

        def run_bwd_staged():  # round-1 sequence: zero + lookup_bwd per lookup + pool_bwd + GEMMs
            gbuf.zero_()
            for c, go in zip(coords, gouts):
                _lib.lookup_bwd(c, go, r, gpyr)
            _lib.pool_bwd(gpyr, H, W)
            return _lib.build_bwd(gpyr[0], f1, f2)

        def autograd_step():  # what training runs: CorrBlock forward + loss.backward() to both fmaps
            cb = CorrBlock(f1g, f2g, num_levels=L, radius=r)
            outs_ = [cb(c) for c in coords]
            torch.autograd.backward(outs_, gouts)
            f1g.grad = None
            f2g.grad = None

    stream = torch.cuda.Stream(device=dev)
    bcast_ms = None
    with torch.cuda.stream(stream):
        if not sharded:  # first call through the public drop-in API (validates the path)
            CorrBlock(f1, f2, num_levels=L, radius=r)(coords[0])
        build_only()
        run_lookups()
        torch.cuda.synchronize()

        # row-sharded, N > 1: the product API for a stream of pairs (eraft_amd.sharded):
        # Fmap2DoubleBuffer.prefetch issues pair k+1's fmap2 broadcast (async, RCCL stream) before
        # pair k's RowShardedCorrBlock is built from the buffer whose broadcast was issued one
        # pair earlier, so the broadcast overlaps the build and the 12 lookups.
        pipe = {"pending": None}
        prefetch = sharded and world > 1 and args.prefetch
        if sharded and world > 1:
            from eraft_amd.sharded import Fmap2DoubleBuffer, RowShardedCorrBlock
        if prefetch:
            dbuf = Fmap2DoubleBuffer(tuple(f2.shape), dev)
            with torch.no_grad():  # the double buffer is inference-only
                pipe["pending"] = dbuf.prefetch(f2 if rank == 0 else None)  # prologue: pair 0's fmap2

        def pair():
            if prefetch:
                cur = pipe["pending"]
                with torch.no_grad():
                    pipe["pending"] = dbuf.prefetch(f2 if rank == 0 else None)
                blk = RowShardedCorrBlock(f1, cur, num_levels=L, radius=r, fmap1_is_slab=True)
                for c in coords:
                    blk(c)
            elif sharded and world > 1:
                # chunked broadcast: chunk k+1 arrives while chunk k's pyramid rows are built
                blk = RowShardedCorrBlock(f1, f2, num_levels=L, radius=r, fmap1_is_slab=True, chunks=args.chunks)
                for c in coords:
                    blk(c)
            elif sharded:  # one rank: the row-slab library calls over all rows
                build_only()
                run_lookups_reused()
            else:
                api_pair()

        # gloo collectives on device tensors go through host copies: not capturable (and a failed
        # capture poisons the stream), so only an RCCL sharded pair is captured
        host_coll = sharded and world > 1 and dist.get_backend() != "nccl"
        launch = "eager" if args.eager or prefetch or host_coll else "hipgraph"
        capture_error = None
        step = pair
        if train:
            step = autograd_step
            try:  # the whole autograd step as one HIP graph (its allocations come from the pool)
                for _ in range(2):
                    autograd_step()
                torch.cuda.synchronize()
                if not args.eager:
                    g_step = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g_step, stream=stream):
                        autograd_step()
                    step = g_step.replay
            except Exception as exc:  # noqa: BLE001 — report and stay eager
                print(f"train: graph capture of the autograd step failed ({exc}); eager", file=sys.stderr)
                capture_error = f"{type(exc).__name__}: {exc}"
                launch = "eager"
                step = autograd_step
        elif launch == "hipgraph":
            try:  # the sharded pair captures its RCCL chunk broadcasts too
                pair()
                torch.cuda.synchronize()
                g_pair = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_pair, stream=stream):
                    pair()
                step = g_pair.replay
            except Exception as exc:  # noqa: BLE001 — report and stay eager
                if not sharded:
                    raise
                print(f"sharded: graph capture failed ({exc}); eager", file=sys.stderr)
                capture_error = f"{type(exc).__name__}: {exc}"
                launch = "eager"
                step = pair
            if sharded and world > 1:
                # every rank must replay the same collectives: one failed capture makes all eager
                ok = torch.tensor([1 if capture_error is None else 0], device=dev, dtype=torch.int32)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if int(ok.item()) == 0 and capture_error is None:
                    capture_error = "another rank's capture failed"
                    launch = "eager"
                    step = pair

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        # the sharded pair holds collectives: every rank replays it the same number of times
        settle(step, fixed=32 if sharded and world > 1 else None)

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        if pipe["pending"] is not None:  # the in-flight broadcast counts inside the timed region
            pipe["pending"].wait()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()

        # the same step with the other build algorithms, and through the public drop-in API
        # (CorrBlock ctor: pyramid + workspace allocation, then 12 __call__s), reported beside
        # `value` — same K steps after W warmups, HIP graphs unless --eager
        alt_values = {}
        if primary and not train and not sharded:
            def timed(fn):
                st = fn
                if launch == "hipgraph":
                    gg = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gg, stream=stream):
                        fn()
                    st = gg.replay
                for _ in range(args.warmup):
                    st()
                torch.cuda.synchronize()
                settle(st)
                a0 = time.perf_counter()
                for _ in range(args.steps):
                    st()
                torch.cuda.synchronize()
                return round(B * args.steps / (time.perf_counter() - a0), 2)

            for nm, bfn in (("fp32", build_fp32), ("f16x3", build_f16x3)):
                if BUILD_ALGO[algo] != nm:
                    alt_values[f"build_{nm}"] = timed(lambda bfn=bfn: (bfn(), run_lookups_reused()))
            alt_values[f"library_calls_{BUILD_ALGO[algo]}"] = timed(lambda: (build_only(), run_lookups_reused()))
            alt_values[f"library_calls_12_outputs_{BUILD_ALGO[algo]}"] = timed(lambda: (build_only(), run_lookups()))

        # per-kernel durations on the launch stream (graph_time_ms)
        build_call_ms = graph_time_ms(build_only, stream)
        if algo != _lib.BUILD_FP32:  # per-kernel: pack + MFMA, each timed alone (kernel-trace comparable)
            pack_ms, mfma_ms = graph_time_ms(build_pack, stream), graph_time_ms(build_mfma, stream)
            build_ms = pack_ms + mfma_ms
        else:
            pack_ms = mfma_ms = None
            build_ms = build_call_ms
        look_ms = graph_time_ms(run_lookups, stream) / iters
        fp32_ms = graph_time_ms(build_fp32, stream, rep=4) if primary and algo != _lib.BUILD_FP32 else None
        x3_ms = graph_time_ms(build_f16x3, stream, rep=4) if primary and algo == _lib.BUILD_BF16X6 else None
        bwd_ms = graph_time_ms(run_bwd_kernels, stream, rep=4) if train else None
        bwd_staged_ms = graph_time_ms(run_bwd_staged, stream, rep=4) if train else None
        bwd_x3_ms = graph_time_ms(run_bwd_f16x3, stream, rep=4) if train and algo == _lib.BUILD_BF16X6 else None
        if sharded and world > 1:  # per-rank broadcast time (eager, events on the stream)
            ts = []
            for _ in range(5):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                dist.broadcast(f2, src=0)
                z.record(stream)
                z.synchronize()
                ts.append(a.elapsed_time(z))
            bcast_ms = sorted(ts)[len(ts) // 2]
            mine = torch.tensor([rank, h0, h1, bcast_ms, build_ms, look_ms], device=dev, dtype=torch.float64)
            allr = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(allr, mine)
            per_rank = [{"rank": int(v[0]), "rows": [int(v[1]), int(v[2])], "broadcast_ms": round(float(v[3]), 4),
                         "build_ms": round(float(v[4]), 4), "lookup_ms": round(float(v[5]), 4)}
                        for v in (t.cpu() for t in allr)]

    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    pairs = B * args.steps * (1 if sharded else world)
    value = pairs / elapsed
    fl = build_flops(B, D, H, W)
    lb = lookup_bytes(B, H, W, L, r)
    bb = build_bytes(B, D, H, W, L)
    if sharded:  # per-rank kernels process the rank's slab (rank 0 owns the largest)
        frac_rows = (h1 - h0) / H
        fl *= frac_rows
        lb *= frac_rows
        lvn = sum((H >> l) * (W >> l) for l in range(L))
        bb = B * D * (h1 - h0 + H) * W * 4 + B * (h1 - h0) * W * lvn * 4
    look_gbs = lb / (look_ms * 1e-3) / 1e9
    hbm_gbs = (bb + iters * lb) / (build_ms + iters * look_ms) / 1e6

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frame-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (randn fmaps, coords_grid + randn flow), resident in HBM",
            "config": {"workload": f"CorrBlock build + {iters} lookups"
                                   f"{' + autograd backward to both fmaps' if train else ''}, {wl_name} "
                                   f"fmaps [{B},{D},{H},{W}], {L} levels, radius {r}",
                       "global_batch": B * (1 if sharded else world), "launch": launch,
                       "parallelism": (f"row-sharded x{world} (query rows of one pair per GPU, fmap2 broadcast "
                                       + ("double-buffered: pair k+1's during pair k)" if prefetch else
                                          f"in {args.chunks} target-row chunks, each chunk's build on arrival)"))
                       if sharded else
                                      f"replicas x{world} (independent frame pairs per GPU)"},
            "build_algo": BUILD_ALGO[algo],
            "build_arith": BUILD_ARITH[algo],
            "roofline": build_roofline(algo, fl, bb, build_ms, build_traffic(wl_name, algo)),
            "roofline_lookup": {"bound": "hbm", "kernel": "lookup_kernel",
                                "achieved": round(look_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": round(look_gbs / PEAK_HBM_GBS, 4),
                                "traffic": traffic(wl_name, "lookup_kernel"),
                                "avg_us": round(look_ms * 1e3, 3), "bytes_per_launch": lb,
                                "ceiling": lookup_ceiling(wl_name, lb, look_ms, traffic(wl_name, "lookup_kernel"))},
            "kernel_timing": "HIP events around 10 back-to-back launches of one kernel in one HIP graph on "
                             "the launch stream, median of 5: the gaps between dependent launches of DIFFERENT "
                             "kernels are not in avg_us (the build's pack -> MFMA boundary is in "
                             "kernel_us.build_call_in_graph); within one run this agrees with rocprofv3's "
                             "kernel trace (profiles/r05l_dsec_kernel_stats.csv vs prof run: MFMA 70.3 vs "
                             "69.2 us median, lookup 5.80 vs 5.59), across boxes it varies by up to 8 %",
            "hbm_gbs_algorithmic": round(hbm_gbs, 1),
        }
        if pack_ms is not None:
            res["roofline"]["kernel_us"] = {PACK_KERNEL[algo]: round(pack_ms * 1e3, 2),
                                            MFMA_KERNEL[algo]: round(mfma_ms * 1e3, 2),
                                            "build_call_in_graph": round(build_call_ms * 1e3, 2)}
        if fp32_ms is not None:  # the fp32-operand MFMA build, beside the default
            res["build_fp32"] = build_roofline(0, fl, bb, fp32_ms, build_traffic(wl_name, 0))
        if x3_ms is not None:  # the narrower f16x3 split (round-3 default), labelled
            res["build_f16x3"] = build_roofline(1, fl, bb, x3_ms, build_traffic(wl_name, 1))
            res["build_f16x3"]["arith"] = BUILD_ARITH[1]
        if alt_values:
            res["alt_values"] = alt_values
            res["alt_values_note"] = ("frame-pairs/s of the same pair (K steps after W warmups and the settle): "
                                      "`value` runs the drop-in CorrBlock (ctor + 12 __call__s, its pyramid and "
                                      "outputs from the allocator, as E-RAFT runs it); build_fp32 / build_f16x3: "
                                      "library calls with the fp32-operand build / the f16x3 split build (narrower "
                                      "than fp32); library_calls_*: the default build through the C-ABI calls "
                                      "with one reused output buffer, and with 12 distinct preallocated outputs "
                                      "(round 3's step: at B16 their 394 MB stream past the MALL)")
        if train:
            res["backward_kernels"] = {
                "phase": f"corr_backward: {iters} lookup backwards in one launch + pool fold into dC + 2 "
                         f"{BUILD_ALGO[_lib.backward_algo(algo)]} split GEMMs (dF1 = dC F2^T, dF2 = F1^T dC, "
                         "split-K with an ordered reduce), library call alone",
                "arith": BWD_ARITH[_lib.backward_algo(algo)],
                "avg_us": round(bwd_ms * 1e3, 2), "gemm_flops": 2 * fl,
                "staged_avg_us": round(bwd_staged_ms * 1e3, 2),
                "staged_phase": f"zero + {iters} lookup_bwd + pool_bwd + GEMMs (round-1 sequence)"}
            if bwd_x3_ms is not None:
                res["backward_kernels"]["f16x3_avg_us"] = round(bwd_x3_ms * 1e3, 2)
                res["backward_kernels"]["f16x3_arith"] = BWD_ARITH[1]
            res["train_step_note"] = ("value times the autograd step through CorrBlock (forward, 12 "
                                      "lookups, loss.backward() to both fmaps), as training runs it; forward "
                                      "build no narrower than fp32 per row, backward GEMMs on the same exact "
                                      "split with one accumulator (build_arith, backward_kernels.arith)")
        if bcast_ms is not None:
            res["sharded_timing"] = {
                "per_rank": per_rank,
                "overlap": ("eraft_amd.sharded.Fmap2DoubleBuffer: pair k+1's broadcast (async, on the "
                            "collective stream) runs during pair k's RowShardedCorrBlock build + lookups"
                            if prefetch else
                            f"fmap2 broadcast in {args.chunks} target-row chunks (all issued async); each "
                            "chunk's pyramid rows are built (corr_build_region) as soon as it has arrived") +
                           "; per-rank broadcast_ms is the whole broadcast timed alone",
                "backend": os.environ.get("ERAFT_AMD_DIST_BACKEND", "nccl")}
        if capture_error is not None:
            res["capture_error"] = capture_error
        if role != "leg" and world == 1 and not args.no_cpu_baseline and wl_name not in CPU_SKIP:
            budget = args.cpu_seconds * (1.0 if primary else 0.5)
            cb = cpu_baseline(wl, budget, train)
            res["cpu_baseline"] = cb
            res["speedup_vs_cpu"] = round(value / cb["value"], 1)
            res["cpu_baseline_1thread"] = cpu_baseline(wl, budget * 0.75, train, threads=1)
        return res
    return None


if __name__ == "__main__":
    main()
