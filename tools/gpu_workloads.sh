#!/bin/bash
# Every bench workload on one GPU box, no CPU baselines (run via gpurun):
#   bash tools/gpu_workloads.sh <tag>   -> gpurun_out/bench_<tag>_<workload>.json
set -o pipefail
TAG=${1:-wl}
mkdir -p gpurun_out
for w in dsec mvsec mvsec_crop hires1280 hires1920; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_$w.json 2> gpurun_out/bench_${TAG}_$w.err || { echo "BENCH $w FAILED"; tail gpurun_out/bench_${TAG}_$w.err; exit 5; }
done
timeout -k 10 200 python bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_train.json 2> gpurun_out/bench_${TAG}_train.err || { echo "BENCH train FAILED"; exit 5; }
timeout -k 10 100 tools/_build/kbench_build 5 mvsec-pad > gpurun_out/kb_${TAG}_mvsec.txt 2>&1 || exit 6
timeout -k 10 200 tools/_build/kbench_build 3 1920x1280 > gpurun_out/kb_${TAG}_1920.txt 2>&1 || exit 6
python3 - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
for w in ["dsec", "mvsec", "mvsec_crop", "hires1280", "hires1920", "train"]:
    d = json.load(open(f"gpurun_out/bench_{tag}_{w}.json"))
    r = d["roofline"]; l = d.get("roofline_lookup", {})
    print(f"{w:11s} {d['value']:10.1f} fps  step {d['ms_per_step']*1e3:8.1f} us  build {r['avg_us']:8.1f} us frac {r['frac']:.3f} "
          f"bind {r.get('binding_floor', {}).get('frac')}  lookup {l.get('avg_us')} us frac {l.get('frac')}")
PY
