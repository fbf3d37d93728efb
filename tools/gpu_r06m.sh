#!/bin/bash
# Round-6 traffic profiles at HEAD (kernel trace + FETCH_SIZE + WRITE_SIZE per workload, summarised
# to gpurun_out/prof_r06m_<w>/pmc.json) and an in-step SQ / TA pass over the train step (the fold).
set -eo pipefail
export TMPDIR=/tmp
for w in dsec train mvsec hires1280; do
  OUT=gpurun_out/prof_r06m_$w
  mkdir -p "$OUT"
  ARGS="--workload $w --no-cpu-baseline --no-workloads --steps 20 --warmup 5"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc2.err"
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc3.err"
  python3 tools/pmc_summary.py "$OUT" --json "$OUT/pmc.json" > "$OUT/summary.txt"
  find "$OUT" -name "*kernel_trace.csv" -delete; find "$OUT" -name "*counter_collection.csv" -delete
  find "$OUT" -name "*agent_info.csv" -delete
  echo "$w done"
done
OUT=gpurun_out/prof_r06m_train_sq
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 bench.py --workload train --no-cpu-baseline --no-workloads --steps 20 --warmup 5 > /dev/null 2> $OUT/pmc.err
python3 tools/sq_summary.py $OUT/pmc > $OUT/summary.txt
find "$OUT" -name "*.csv" -delete
echo sq done
