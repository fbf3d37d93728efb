#!/bin/bash
# Kernel trace of the train step (fold with the general separable form).  bash tools/gpu_r05zb.sh
set -eo pipefail
mkdir -p gpurun_out/r05zb
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05zb/trace -o run --output-format csv -- python3 bench.py --workload train --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/r05zb/bench_trace.json 2> gpurun_out/r05zb/trace.err
echo trace done
