#!/bin/bash
# bf16x6 pack: records per wave (kbench_build, interleaved rounds) at DSEC / train / MVSEC.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g
for sh in dsec train mvsec-pad; do
  timeout -k 10 240 ./tools/_build/kbench_build 10 $sh "pack only" > gpurun_out/r06g/kb_$sh.txt 2>&1 || { echo "$sh failed"; tail -5 gpurun_out/r06g/kb_$sh.txt; exit 3; }
  echo "$sh done"
done
