"""Summarise rocprofv3 outputs of tools/profile.sh: per-kernel average duration and PMC
counters (averaged per dispatch) for the corr kernels.

    python tools/pmc_summary.py gpurun_out/prof_<tag>                 # text
    python tools/pmc_summary.py gpurun_out/prof_<tag> --json out.json # + machine-readable
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("lookup_conv_bwd_dw_kernel", "lookup_conv_bwd_dlk_kernel", "lookup_conv_bwd_reduce_kernel", "lookup_conv_kernel", "bf16_pack_kernel", "corr_build_bf16_kernel", "lookup_bwd_fold_kernel", "pool_fold_max_kernel", "rowmax2_kernel", "corr_build_split_kernel", "corr_build_split_ring_kernel", "split_pack_reg_kernel", "split_pack_wide_kernel", "split_pack_kernel",
           "corr_build_kernel", "lookup_bwd_kernel", "lookup_kernel", "split_gemm_kernel", "gemm_kernel",
           "splitk_reduce_kernel", "pool_bwd_kernel", "pool2x2_kernel", "split_convert_rows_kernel",
           "split_convert_cols_kernel", "absmax_kernel", "split_gemm_f32_kernel", "colmax_reduce_kernel")


# Kernels whose template instantiations are reported apart (e.g. the f16x3 and bf16x6 GEMMs).
BY_TEMPLATE = ("split_gemm_f32_kernel",)


def short(name):
    for k in KERNELS:
        if k in name:
            if k in BY_TEMPLATE and k + "<" in name:
                i = name.index(k + "<") + len(k)
                return k + name[i:name.index(">", i) + 1]
            return k
    return None


def collect(d):
    out = {"kernels": defaultdict(dict)}
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            s = short(row["Name"])
            if s:
                out["kernels"][s].update(calls=int(row["Calls"]), avg_us=float(row["AverageNs"]) / 1e3,
                                         min_us=float(row["MinNs"]) / 1e3, max_us=float(row["MaxNs"]) / 1e3)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        acc = defaultdict(lambda: defaultdict(list))
        for row in csv.DictReader(open(f)):
            s = short(row.get("Kernel_Name", ""))
            if s:
                acc[s][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, cs in acc.items():
            for c, v in cs.items():
                out["kernels"][k][c] = sum(v) / len(v)
    out["kernels"] = dict(out["kernels"])
    return out


def main(d, js=None):
    res = collect(d)
    for k, v in res["kernels"].items():
        print(f"{k}:")
        for c, x in sorted(v.items()):
            print(f"    {c:28s} {x:.6g}")
    if js:
        res["source"] = d
        res["note"] = ("FETCH_SIZE / WRITE_SIZE in kB per dispatch (rocprofv3, separate --pmc passes); "
                       "gfx950 FETCH_SIZE counts half the bytes of 16-B/lane streaming reads")
        with open(js, "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--json" else None)
