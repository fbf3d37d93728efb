#!/bin/bash
# Round-4 GPU steps (run via gpurun): bash tools/gpu_r04.sh <tag> <step>...
#   kb:<shape>    build kbench (tools/_build/kbench_build) at one shape
#   t:<expr>      pytest -m gpu -k <expr>
#   tests         the whole GPU suite
#   bench:<args>  bench.py with args (commas -> spaces)
set -o pipefail
TAG=${1:-a}; shift || true
NB=0
mkdir -p gpurun_out
export TMPDIR=/tmp
for STEP in "$@"; do
  case "$STEP" in
    kb:*) SH=${STEP#kb:}
      timeout -k 10 180 ./tools/_build/kbench_build 20 $SH > gpurun_out/kb_${TAG}_$SH.txt 2>&1 || { echo "kbench $SH failed"; tail -5 gpurun_out/kb_${TAG}_$SH.txt; exit 3; }
      grep -E "median|DIFFER|identical|scale 1 " gpurun_out/kb_${TAG}_$SH.txt ;;
    t:*) K=${STEP#t:}
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread -k "$K" > gpurun_out/t_${TAG}.txt 2>&1; rc=$?
      tail -30 gpurun_out/t_${TAG}.txt; [ $rc -eq 0 ] || exit 4 ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_${TAG}.txt 2>&1; rc=$?
      tail -15 gpurun_out/tests_${TAG}.txt; [ $rc -eq 0 ] || exit 5 ;;
    bench:*) A=${STEP#bench:}; A=${A//,/ }; NB=$((NB+1)); OUT=gpurun_out/bench_${TAG}_$NB
      timeout -k 10 300 python -u bench.py $A > $OUT.json 2> $OUT.err; rc=$?
      tail -c 1500 $OUT.json; echo; [ $rc -eq 0 ] || { tail -20 $OUT.err; exit 6; } ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo done
