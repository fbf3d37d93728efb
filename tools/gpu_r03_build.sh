#!/bin/bash
# Round-3 build-kernel A/B on the GPU box (run via gpurun): bash tools/gpu_r03_build.sh <tag> [shapes...]
set -o pipefail
TAG=${1:-a}; shift || true
mkdir -p gpurun_out
export TMPDIR=/tmp
for SH in "${@:-dsec}"; do
  timeout -k 10 120 ./tools/_build/kbench_build 20 $SH > gpurun_out/kb_${TAG}_$SH.txt 2>&1 || { echo "kbench $SH failed"; tail -5 gpurun_out/kb_${TAG}_$SH.txt; exit 3; }
  grep -v "^$" gpurun_out/kb_${TAG}_$SH.txt | grep -E "median|DIFFER|identical|scale 1 " 
done
echo done
