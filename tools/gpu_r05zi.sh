#!/bin/bash
# Several query groups per fold workgroup: backward GPU tests, kbench_bwd, a TA/TD PMC pass,
# train bench.   bash tools/gpu_r05zi.sh
set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or autograd or config4 or golden or sharded or fold" -s > gpurun_out/r05zi_tests.txt 2>&1
echo tests done
timeout -k 10 200 ./tools/_build/kbench_bwd 10 > gpurun_out/r05zi_kbench_bwd.txt 2>&1
echo kbench done
bash tools/gpu_fold_pmc2.sh r05zi "SEP G=4 T=12, no maxima" "SEP G=2 T=12, no maxima"
timeout -k 10 300 python3 -u bench.py --workload train > gpurun_out/r05zi_bench_train.json 2> gpurun_out/r05zi_bench_train.err
echo bench done
