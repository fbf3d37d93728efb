#!/bin/bash
# Backward + sharded checks on the GPU box (run via gpurun):  bash tools/gpu_round2.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "multi_and_fold or matches_staged or fused_backward or training_shape or determinism or build_bwd or backward_matches_reference or slab_backward" \
  tests/test_configs.py::test_config4_train_b8_d256_forward_backward tests/test_sharded.py > gpurun_out/t_bwd.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sw -o run -- python3 tools/bwd_sweep.py grid > gpurun_out/sw.log 2>&1 || exit 4
timeout -k 10 200 python bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_train.json 2> gpurun_out/b_train.err || exit 5
ERAFT_AMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload hires1280 --sharded --steps 5 --warmup 2 \
  --no-cpu-baseline > gpurun_out/b_shard2.json 2> gpurun_out/b_shard2.err || exit 6
echo done
