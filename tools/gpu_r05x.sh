#!/bin/bash
# LDS-staged bf16x6 pack: build / pack / region / backward-inf GPU tests, then old and new
# kbench_build interleaved (pack only, pack + MFMA) at DSEC, MVSEC and train.
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "bf16x6 or build or region or pack or configs or inf or sharded" > gpurun_out/r05x_tests.txt 2>&1
echo tests done
for sh in dsec mvsec-pad train; do
  for v in base new base new; do
    b=tools/_build/kbench_build; [ $v = base ] && b=${b}_base
    echo "== $v $sh" >> gpurun_out/r05x_kbench_build.txt
    timeout -k 10 150 $b 5 $sh bf16x6 >> gpurun_out/r05x_kbench_build.txt 2>&1
  done
done
echo kbench done
