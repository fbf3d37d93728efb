#!/bin/bash
# Round-3 full GPU pass (run via gpurun): GPU tests + smoke, every bench workload, the DSEC bench
# with CPU baselines and its rocprofv3 trace / PMC passes.   bash tools/gpu_r03_full.sh <tag>
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/gpu_tests_$TAG.log | head; tail -5 gpurun_out/gpu_tests_$TAG.log; exit 3; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "SMOKE FAILED"; cat gpurun_out/smoke_$TAG.log; exit 4; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/gpu_workloads.sh $TAG || exit 5
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "BENCH FAILED"; tail gpurun_out/bench_$TAG.err; exit 6; }
cat gpurun_out/bench_$TAG.json
bash tools/profile.sh $TAG || { echo "PROFILE FAILED"; exit 7; }
echo done
