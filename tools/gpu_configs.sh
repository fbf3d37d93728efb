#!/bin/bash
# All BASELINE configs on one GPU box (run via gpurun):  bash tools/gpu_configs.sh <tag>
# GPU tests, then bench.py per workload -> gpurun_out/bench_<tag>_<workload>.json
set -o pipefail
TAG=${1:-cfg}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 3; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 200 python bench.py > gpurun_out/bench_${TAG}_dsec.json 2> gpurun_out/bench_${TAG}_dsec.err || { echo "BENCH dsec FAILED"; tail gpurun_out/bench_${TAG}_dsec.err; exit 5; }
timeout -k 10 200 python bench.py --workload train --steps 20 > gpurun_out/bench_${TAG}_train.json 2> gpurun_out/bench_${TAG}_train.err || { echo "BENCH train FAILED"; tail gpurun_out/bench_${TAG}_train.err; exit 5; }
timeout -k 10 200 python bench.py --workload mvsec --steps 20 --cpu-seconds 10 > gpurun_out/bench_${TAG}_mvsec.json 2> gpurun_out/bench_${TAG}_mvsec.err || { echo "BENCH mvsec FAILED"; tail gpurun_out/bench_${TAG}_mvsec.err; exit 5; }
timeout -k 10 200 python bench.py --workload hires1280 --sharded --steps 10 --no-cpu-baseline > gpurun_out/bench_${TAG}_hires1280.json 2> gpurun_out/bench_${TAG}_hires1280.err || { echo "BENCH hires FAILED"; tail gpurun_out/bench_${TAG}_hires1280.err; exit 5; }
for w in dsec train mvsec hires1280; do echo "== $w"; cat gpurun_out/bench_${TAG}_$w.json; done
