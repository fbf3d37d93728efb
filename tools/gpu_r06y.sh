#!/bin/bash
# Traffic profile of config 5's 1920x1280 size at HEAD (kernel trace + FETCH_SIZE + WRITE_SIZE,
# summarised to gpurun_out/prof_r06y_hires1920/pmc.json) for bench.py's roofline traffic.
set -eo pipefail
export TMPDIR=/tmp
for w in hires1920; do
  OUT=gpurun_out/prof_r06y_$w
  mkdir -p "$OUT"
  ARGS="--workload $w --no-cpu-baseline --no-workloads --steps 10 --warmup 3"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc2.err"
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc3.err"
  python3 tools/pmc_summary.py "$OUT" --json "$OUT/pmc.json" > "$OUT/summary.txt"
  find "$OUT" -name "*kernel_trace.csv" -delete; find "$OUT" -name "*counter_collection.csv" -delete
  find "$OUT" -name "*agent_info.csv" -delete
  echo "$w done"
  cat "$OUT/summary.txt" | head -30
done
