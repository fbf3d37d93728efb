"""bench.py's measurement arithmetic on CPU: the algorithmic counts SURVEY §8(d) quotes per
config, the roofline / ceiling formulas, the committed PMC traffic it reads, and the workload
table the driver's default run walks (no GPU: nothing here launches a kernel)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_algorithmic_counts_match_survey():
    # DSEC build 11.80 GFLOP / 132.1 MB, lookup 13.94 MB per call;
    # MVSEC 36x44 B16 20.55 GFLOP, lookup 73.6 MB; train B8 36x48 12.23 GFLOP, lookup 40.1 MB
    B, D, H, W, L, r, _ = bench.WORKLOADS["dsec"]
    assert bench.build_flops(B, D, H, W) / 1e9 == pytest.approx(11.80, abs=0.005)
    assert bench.build_bytes(B, D, H, W, L) / 1e6 == pytest.approx(132.1, abs=0.05)
    assert bench.lookup_bytes(B, H, W, L, r) / 1e6 == pytest.approx(13.94, abs=0.005)
    B, D, H, W, L, r, _ = bench.WORKLOADS["mvsec"]
    assert bench.build_flops(B, D, H, W) / 1e9 == pytest.approx(20.55, abs=0.005)
    assert bench.lookup_bytes(B, H, W, L, r) / 1e6 == pytest.approx(73.6, abs=0.05)
    B, D, H, W, L, r, _ = bench.WORKLOADS["train"]
    assert bench.build_flops(B, D, H, W) / 1e9 == pytest.approx(12.23, abs=0.005)
    assert bench.lookup_bytes(B, H, W, L, r) / 1e6 == pytest.approx(40.1, abs=0.05)
    # per query: L (2r+2)^2 + L (2r+1)^2 floats + the 8 B of coords
    assert bench.lookup_bytes(1, 1, 1, 4, 4) == 4 * 100 * 4 + 4 * 81 * 4 + 8


def test_workload_table_covers_the_baseline_configs():
    for wl in bench.EXTRA_WORKLOADS:
        assert wl in bench.WORKLOADS or wl == "e2e", wl
    # configs 2-5 beside the DSEC value: train (4), mvsec (3), both config-5 sizes, e2e (2)
    assert set(bench.EXTRA_WORKLOADS) == {"train", "mvsec", "hires1280", "hires1920", "e2e"}
    assert bench.WORKLOADS["hires1920"][2:4] == (160, 240)  # 1920x1280 / 8
    assert bench.WORKLOADS["hires1280"][2:4] == (120, 160)


def test_build_roofline_prices_the_executed_pipe():
    B, D, H, W, L, _, _ = bench.WORKLOADS["dsec"]
    fl, bb = bench.build_flops(B, D, H, W), bench.build_bytes(B, D, H, W, L)
    t_ms = 0.075
    rf = bench.build_roofline(2, fl, bb, t_ms, None)  # bf16x6: 6 executed products per fp32 one
    assert rf["bound"] == "mfma" and rf["peak"] == bench.PEAK_F16_MFMA_TFLOPS
    assert rf["achieved"] == pytest.approx(6 * fl / (t_ms * 1e-3) / 1e12, rel=1e-3)
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], abs=1e-4)
    assert rf["fp32_equivalent_tflops"] == pytest.approx(fl / (t_ms * 1e-3) / 1e12, rel=1e-3)
    r0 = bench.build_roofline(0, fl, bb, t_ms, None)  # the fp32-operand build: fp32 MFMA peak
    assert r0["peak"] == bench.PEAK_FP32_MFMA_TFLOPS
    assert r0["achieved"] == pytest.approx(fl / (t_ms * 1e-3) / 1e12, rel=1e-3)


def test_lookup_ceiling_binds_the_lower_bound():
    lb = bench.lookup_bytes(1, 60, 80, 4, 4)
    c = bench.lookup_ceiling("dsec", lb, 0.0055, 2 * lb)
    floor = c["latency_floor"]["frac"]
    gran = c["line_granularity"]["frac"]
    assert floor == pytest.approx(lb / (bench.LOOKUP_NOLOAD_NOSTORE_US["dsec"] * 1e-6) / 1e9 / bench.PEAK_HBM_GBS,
                                  abs=1e-4)
    assert gran == pytest.approx(0.5 * bench.ACHIEVABLE_HBM_GBS / bench.PEAK_HBM_GBS, abs=1e-4)
    assert c["binding"] == ("latency_floor" if floor < gran else "line_granularity")
    frac = lb / 0.0055e-3 / 1e9 / bench.PEAK_HBM_GBS
    assert c["frac_of_ceiling"] == pytest.approx(frac / min(floor, gran), abs=1e-3)
    # no floor measured and no PMC pass: no ceiling claimed
    assert bench.lookup_ceiling("mvsec_crop", lb, 0.03, None) == {}
    # every workload the default line measures has a measured floor
    assert all(w in bench.LOOKUP_NOLOAD_NOSTORE_US for w in bench.EXTRA_WORKLOADS if w != "e2e")


def test_traffic_reads_the_newest_committed_pmc_pass():
    t = bench.traffic("dsec", "lookup_kernel")
    assert t is not None and t > bench.lookup_bytes(1, 60, 80, 4, 4)  # line granularity: > algorithmic
    bt = bench.build_traffic("dsec", 2)
    assert bt is not None and bt >= bench.build_bytes(1, 256, 60, 80, 4)  # pyramid + packed operands
    assert bench.traffic("no_such_workload", "lookup_kernel") is None
