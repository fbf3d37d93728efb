#!/bin/bash
# Fold: upstream gradients two lookups ahead (PD2) vs one; A/B HEAD vs working tree kbench_bwd, warm and cold.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06t
mkdir -p $OUT
for r in 1 2; do
  for b in kbench_bwd_old kbench_bwd; do
    echo "== $b round $r" >> $OUT/ab.txt
    timeout -k 10 150 ./tools/_build/$b 8 >> $OUT/ab.txt 2>&1 || { echo "$b failed"; exit 3; }
  done
done
grep -E "==|check|LEAN" $OUT/ab.txt
