"""Per-kernel PMC table from tools/pmc_kbench.sh output (gpurun_out/pk)."""
import collections, csv, glob, re, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pk"
def short(k):
    m = re.search(r"(corr_build_split\w*|corr_build_kernel|split_pack_wide_kernel|split_pack_kernel|lookup\w*kernel)", k)
    t = re.findall(r"Li(\d+)E", k)
    return (m.group(1) if m else k[:30]) + ("<" + ",".join(t) + ">" if t else "")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
for f in glob.glob(d + "/tr/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(agg):
    if "fill" in k.lower() or "maxdiff" in k or "rocclr" in k: continue
    ds = sorted(dur.get(k, [0]))
    print(f"{k}  median {ds[len(ds)//2]:.1f} us  n={len(ds)}")
    for c, v in sorted(agg[k].items()):
        print(f"    {c:28s} {sum(v)/len(v):.5g}")
