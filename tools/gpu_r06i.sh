#!/bin/bash
# Fold: LEAN warm / cold and the L2 warm-up variant (kbench_bwd), two rounds.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06i
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 ./tools/_build/kbench_bwd 8 >> $OUT/kb.txt 2>&1 || { echo "kbench failed"; tail -5 $OUT/kb.txt; exit 3; }
done
echo done
