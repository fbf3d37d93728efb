#!/bin/bash
# Quad-coalesced gradient loads in the fold: backward GPU tests, kbench_bwd, a TA/TD PMC pass,
# train bench.   bash tools/gpu_r05zh.sh
set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or autograd or config4 or golden or sharded or fold" -s > gpurun_out/r05zh_tests.txt 2>&1
echo tests done
timeout -k 10 200 ./tools/_build/kbench_bwd 10 > gpurun_out/r05zh_kbench_bwd.txt 2>&1
echo kbench done
bash tools/gpu_fold_pmc2.sh r05zh "SEP full T=12"
timeout -k 10 300 python3 -u bench.py --workload train > gpurun_out/r05zh_bench_train.json 2> gpurun_out/r05zh_bench_train.err
echo bench done
