#!/bin/bash
# Fold: backward parity tests, then A/B (HEAD kernel vs working tree, interleaved) + LDS PMC.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or config4 or fold or staged or autograd" > gpurun_out/r06c/tests.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/r06c/tests.txt; exit 2; }
tail -2 gpurun_out/r06c/tests.txt
bash tools/gpu_r06b.sh r06c
