#!/bin/bash
# Fold prefetching two lookups ahead: full GPU suite,
# kbench_bwd, train bench, train kernel trace.   bash tools/gpu_r05zp.sh
set -eo pipefail
mkdir -p gpurun_out/r05zp
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or autograd or config4 or golden or sharded or fold" > gpurun_out/r05zp_tests.txt 2>&1
echo tests done
timeout -k 10 200 ./tools/_build/kbench_bwd 10 > gpurun_out/r05zp_kbench_bwd.txt 2>&1
echo kbench done
timeout -k 10 300 python3 -u bench.py --workload train > gpurun_out/r05zp_bench_train.json 2> gpurun_out/r05zp_bench_train.err
echo bench done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05zp/trace -o run --output-format csv -- python3 bench.py --workload train --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/r05zp/bench_trace.json 2> gpurun_out/r05zp/trace.err
echo trace done
