"""Median per-dispatch PMC counters per corr kernel from one rocprofv3 --pmc output directory.

    python tools/sq_summary.py <dir> > summary.txt
"""
import collections
import csv
import glob
import statistics
import sys

NAMES = ("lookup_bwd_fold_kernel", "split_gemm_f32_kernel", "lookup_kernel", "corr_build_bf16_kernel",
         "bf16_pack_kernel", "splitk_reduce_vec4_kernel")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for n in NAMES:
            if n + "<" in r["Kernel_Name"] or n + "(" in r["Kernel_Name"]:
                agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, d in agg.items():
    print(n, " ".join(f"{c}={statistics.median(v):.4g}" for c, v in sorted(d.items())))
