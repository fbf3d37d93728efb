#!/bin/bash
# bf16x6 build tile orders / L2 tile-group sizes at every size (kbench_build, interleaved rounds).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06d
for sh in dsec train mvsec-pad 1280x960 1920x1280; do
  timeout -k 10 240 ./tools/_build/kbench_build 6 $sh "bf16x6 mfma o" > gpurun_out/r06d/kb_$sh.txt 2>&1 || { echo "$sh failed"; tail -5 gpurun_out/r06d/kb_$sh.txt; exit 3; }
  echo "$sh done"
done
