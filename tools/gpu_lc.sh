#!/bin/bash
# lookup_conv (f16x3) checks + timing on the GPU box (run via gpurun):  bash tools/gpu_lc.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "lookup_conv" \
  tests/test_e2e.py > gpurun_out/t_lc.log 2>&1 || exit 3
timeout -k 10 200 python tools/kbench_aux.py > gpurun_out/kb_aux.json 2> gpurun_out/kb_aux.err || exit 4
echo done
