#!/bin/bash
# Window row stride 16 (26.6 KB per 32-query workgroup: 6 per CU): lookup / conv GPU tests, kbench_lookup
# (QB 16 / 28 / 32), same-box A/B of the DSEC and train forward steps against HEAD's library.
#   bash tools/gpu_r05zv.sh
set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "lookup or golden or conv or config or corr_block or smoke or sharded" > gpurun_out/r05zv_tests.txt 2>&1
echo tests done
timeout -k 10 300 ./tools/_build/kbench_lookup 20 > gpurun_out/r05zv_kbench_lookup.txt 2>&1
echo kbench done
timeout -k 10 300 python3 -u tools/ab_step.py dsec 9 > gpurun_out/r05zv_ab_dsec.txt 2>&1
timeout -k 10 300 python3 -u tools/ab_step.py train 9 > gpurun_out/r05zv_ab_train.txt 2>&1
timeout -k 10 300 python3 -u tools/ab_step.py mvsec 9 > gpurun_out/r05zv_ab_mvsec.txt 2>&1
echo ab done
