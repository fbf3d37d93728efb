#!/bin/bash
# Traffic profiles for every non-default workload (run via gpurun): per workload a kernel trace
# and the FETCH_SIZE / WRITE_SIZE passes, summarised to gpurun_out/prof_<tag>_<w>/pmc.json
# (copy to profiles/<tag>_<w>_pmc.json: bench.py reads the newest one for its traffic fields).
#   bash tools/gpu_pmc_all.sh <tag>
set -eo pipefail
TAG=${1:-pmc}
export TMPDIR=/tmp
for w in train mvsec mvsec_crop hires1280 hires1920; do
  OUT=gpurun_out/prof_${TAG}_$w
  mkdir -p "$OUT"
  ARGS="--workload $w --no-cpu-baseline --steps 20 --warmup 5"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc2.err"
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc3.err"
  python3 tools/pmc_summary.py "$OUT" --json "$OUT/pmc.json" > "$OUT/summary.txt"
  echo "$w done"
done
