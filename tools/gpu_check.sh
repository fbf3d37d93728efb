#!/bin/bash
# One GPU-box pass (run via gpurun): parity tests, smoke, bench (JSON), rocprofv3 profile.
#   tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift || true
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 3; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "SMOKE FAILED"; cat gpurun_out/smoke_$TAG.log; exit 4; }
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "BENCH FAILED"; tail gpurun_out/bench_$TAG.err; exit 5; }
cat gpurun_out/bench_$TAG.json
bash tools/profile.sh $TAG "$@" || { echo "PROFILE FAILED"; exit 6; }
cat gpurun_out/prof_$TAG/summary.txt
