#!/bin/bash
# Lookup ablations at config 5's 1920x1280 size (the latency floor bench.py quotes for hires1920).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06za
mkdir -p $OUT
timeout -k 10 240 tools/_build/kbench_lookup 20 1920x1280 > $OUT/kbench_lookup_1920.txt 2>&1 || { echo kbench failed; tail -20 $OUT/kbench_lookup_1920.txt; exit 2; }
cat $OUT/kbench_lookup_1920.txt
