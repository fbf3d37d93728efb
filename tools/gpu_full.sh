#!/bin/bash
# Full validation + measurement pass (run via gpurun): the GPU test suite, smoke(), then
# tools/gpu_r05.sh's bench lines, gloo rehearsal and profiles.   bash tools/gpu_full.sh <tag> [prof workloads]
set -eo pipefail
TAG=${1:-full}
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/${TAG}_tests.txt 2>&1
echo "tests done"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
echo "smoke done"
PROF="${2:-dsec train}" bash tools/gpu_r05.sh ${TAG}
