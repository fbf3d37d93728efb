#!/bin/bash
# Round-3 GPU pass (run via gpurun): selected GPU tests, then the build kbench.
#   bash tools/gpu_r03_check.sh <tag> <pytest -k expr> [kbench shapes...]
set -o pipefail
TAG=${1:-a}; K=${2:-}; shift 2 || true
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "$K" > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -4 gpurun_out/t_$TAG.log; grep -E "FAIL|Error" gpurun_out/t_$TAG.log | head -20
  [ $rc -eq 0 ] || exit 3
fi
for SH in "$@"; do
  timeout -k 10 150 ./tools/_build/kbench_build 20 $SH > gpurun_out/kb_${TAG}_$SH.txt 2>&1 || { echo "kbench $SH failed"; tail -5 gpurun_out/kb_${TAG}_$SH.txt; exit 4; }
  grep -E "median|DIFFER|identical|scale 1 " gpurun_out/kb_${TAG}_$SH.txt
done
echo done
