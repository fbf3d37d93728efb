#!/bin/bash
# bf16x6 build: 8-wave workgroups (256 queries per target patch) vs the 4-wave default.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06k
for sh in dsec train mvsec-pad 1280x960; do
  timeout -k 10 240 ./tools/_build/kbench_build 8 $sh "mfma o" > gpurun_out/r06k/kb_$sh.txt 2>&1 || { echo "$sh failed"; tail -5 gpurun_out/r06k/kb_$sh.txt; exit 3; }
  echo "$sh done"
done
