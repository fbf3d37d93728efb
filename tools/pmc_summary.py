"""Summarise rocprofv3 outputs of tools/profile.sh: per-kernel average duration and PMC
counters (per dispatch), for the corr kernels.   python tools/pmc_summary.py gpurun_out/prof_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    for k in ("corr_build_kernel", "lookup_bwd_kernel", "lookup_kernel", "gemm_kernel",
              "splitk_reduce_kernel", "pool_bwd_kernel", "pool2x2_kernel"):
        if k in name:
            return k + ("<" + name.split("<", 1)[1].split(">")[0] + ">" if "<" in name else "")
    return None


def main(d):
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    for f in stats:
        print("== kernel stats", f)
        for row in csv.DictReader(open(f)):
            s = short(row["Name"])
            if s:
                print(f"  {s:40s} calls {row['Calls']:>6s} avg {float(row['AverageNs'])/1e3:9.2f} us"
                      f"  min {float(row['MinNs'])/1e3:9.2f}  max {float(row['MaxNs'])/1e3:9.2f}")
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        acc = defaultdict(lambda: defaultdict(list))
        for row in csv.DictReader(open(f)):
            s = short(row.get("Kernel_Name", ""))
            if s:
                acc[s][row["Counter_Name"]].append(float(row["Counter_Value"]))
        print("== pmc", f)
        for k, cs in acc.items():
            print("  ", k, "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main(sys.argv[1])
