#!/bin/bash
# Final round-6 validation at HEAD: full GPU suite, default bench (DSEC + workloads), DSEC and train kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zc
mkdir -p $OUT
timeout -k 10 420 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $OUT/tests.txt 2>&1 || { echo tests failed; tail -30 $OUT/tests.txt; exit 2; }
tail -2 $OUT/tests.txt
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 3; }
echo bench done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/dsec_trace -o run --output-format csv -- python3 bench.py --no-workloads --no-cpu-baseline --steps 200 --warmup 10 > $OUT/dsec_trace.json 2> $OUT/dsec_trace.err || { echo trace failed; exit 4; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/train_trace -o run --output-format csv -- python3 bench.py --workload train --no-cpu-baseline --steps 50 --warmup 10 > $OUT/train_trace.json 2> $OUT/train_trace.err || { echo trace failed; exit 5; }
echo traces done
