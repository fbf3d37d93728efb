#!/bin/bash
# fp32-operand build with paired-lane level-0 stores: build GPU tests, then old and new
# kbench_build interleaved (the f32 variants) at DSEC and train.
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "fp32 or FP32 or build or configs or golden" > gpurun_out/r05y_tests.txt 2>&1
echo tests done
for sh in dsec train; do
  for v in base new base new; do
    b=tools/_build/kbench_build; [ $v = base ] && b=${b}_base
    echo "== $v $sh" >> gpurun_out/r05y_kbench_build.txt
    timeout -k 10 150 $b 5 $sh f32 >> gpurun_out/r05y_kbench_build.txt 2>&1
  done
done
echo kbench done
