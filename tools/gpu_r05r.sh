#!/bin/bash
# f16x3 tile-block epilogue + tile order 3: GPU tests of the builds, then old / new kbench_build
# interleaved at DSEC and train.   bash tools/gpu_r05r.sh
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "f16x3 or split or F16X3 or build or configs" > gpurun_out/r05r_tests.txt 2>&1
echo tests done
for sh in dsec train; do
  for v in base new base new; do
    b=tools/_build/kbench_build; [ $v = base ] && b=${b}_base
    echo "== $v $sh" >> gpurun_out/r05r_kbench_build.txt
    timeout -k 10 150 $b 5 $sh >> gpurun_out/r05r_kbench_build.txt 2>&1
  done
done
echo kbench done
