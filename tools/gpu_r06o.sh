#!/bin/bash
# Lookup without the first barrier (anchors from the gather wave's own lanes): kbench A/B, GPU suite.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06o
mkdir -p $OUT
timeout -k 10 240 tools/_build/kbench_lookup 30 > $OUT/kbench_lookup.txt 2>&1 || { echo kbench failed; tail -20 $OUT/kbench_lookup.txt; exit 2; }
grep -E "!!|prod launch|r5 order|QB32  |QB16  |QB32 tight  " $OUT/kbench_lookup.txt
timeout -k 10 420 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $OUT/tests.txt 2>&1 || { echo tests failed; tail -30 $OUT/tests.txt; exit 3; }
tail -2 $OUT/tests.txt
