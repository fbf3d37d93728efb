#!/bin/bash
# Full forward (config 2): MIOpen algorithm search on / off, and a kernel trace of the default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06u
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/e2e_ab.py --steps 20 --warmup 3 > $OUT/e2e_ab.txt 2>&1 || { echo e2e_ab failed; tail -20 $OUT/e2e_ab.txt; exit 2; }
cat $OUT/e2e_ab.txt | grep -v amdgpu.ids
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/e2e_trace -o run --output-format csv -- python3 bench.py --workload e2e --no-cpu-baseline --steps 10 --warmup 2 > $OUT/e2e_trace.json 2> $OUT/e2e_trace.err || { echo trace failed; exit 4; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r06u/e2e_trace/run_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms', tot/1e6)
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% {int(r['Calls']):6d} {r['Name'][:110]}")
PY
