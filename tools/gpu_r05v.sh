#!/bin/bash
# Separable fold: the backward / autograd / config GPU tests, then tools/kbench_bwd (exact and
# separable kernels in one binary), and the train bench line.   bash tools/gpu_r05v.sh
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or autograd or config4 or golden or lookup_conv or sharded or fold" -s > gpurun_out/r05v_tests.txt 2>&1
echo tests done
timeout -k 10 200 ./tools/_build/kbench_bwd 10 > gpurun_out/r05v_kbench_bwd.txt 2>&1
echo kbench done
timeout -k 10 300 python3 -u bench.py --workload train > gpurun_out/r05v_bench_train.json 2> gpurun_out/r05v_bench_train.err
echo bench done
