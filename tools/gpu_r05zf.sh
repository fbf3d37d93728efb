#!/bin/bash
# General separable form for irregular fold windows: backward / autograd GPU tests, kbench_bwd,
# train bench.   bash tools/gpu_r05zf.sh
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or autograd or config4 or golden or sharded or fold" -s > gpurun_out/r05zf_tests.txt 2>&1
echo tests done
timeout -k 10 200 ./tools/_build/kbench_bwd 10 > gpurun_out/r05zf_kbench_bwd.txt 2>&1
echo kbench done
timeout -k 10 300 python3 -u bench.py --workload train > gpurun_out/r05zf_bench_train.json 2> gpurun_out/r05zf_bench_train.err
echo bench done
