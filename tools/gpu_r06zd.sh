#!/bin/bash
# Multi-rank rehearsal at HEAD on the one-GPU box (gloo: ranks share the GPU): --gpus 2 (DSEC
# replicas + the sharded 1280x960 leg) and --gpus 4 --workload hires1280 --sharded.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zd
mkdir -p $OUT
ERAFT_AMD_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_dsec_gpus2_gloo.json 2> $OUT/gpus2.err || { echo gpus2 failed; tail -20 $OUT/gpus2.err; exit 2; }
echo gpus2 done
ERAFT_AMD_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 4 --workload hires1280 --sharded --steps 10 --warmup 3 > $OUT/bench_hires1280_sharded4_gloo.json 2> $OUT/gpus4.err || { echo gpus4 failed; tail -20 $OUT/gpus4.err; exit 3; }
echo gpus4 done
