#!/bin/bash
# Lookup A/B: early gather vs barrier variants and the r5 order, with ablations.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06s
mkdir -p $OUT
timeout -k 10 240 tools/_build/kbench_lookup 30 > $OUT/kbench_lookup.txt 2>&1 || { echo kbench failed; tail -20 $OUT/kbench_lookup.txt; exit 2; }
grep -E "!!|dsec|train  " $OUT/kbench_lookup.txt
