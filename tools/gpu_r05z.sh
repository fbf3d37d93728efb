#!/bin/bash
# Launch floor under HIP runtime settings: the empty / store kernels in a graph (kbench_floor)
# and the DSEC bench step, with the default settings and with HIP_FORCE_DEV_KERNARG=1.
set -eo pipefail
mkdir -p gpurun_out
for kv in default HIP_FORCE_DEV_KERNARG=1 HIP_FORCE_DEV_KERNARG=0; do
  echo "== $kv" >> gpurun_out/r05z_floor.txt
  if [ $kv = default ]; then timeout -k 10 60 ./tools/_build/kbench_floor >> gpurun_out/r05z_floor.txt 2>&1
  else env $kv timeout -k 10 60 ./tools/_build/kbench_floor >> gpurun_out/r05z_floor.txt 2>&1; fi
done
echo floor done
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/r05z_bench_dsec_default.json 2> gpurun_out/r05z_bench.err
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/r05z_bench_dsec_devkernarg.json 2>> gpurun_out/r05z_bench.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/r05z_bench_dsec_default2.json 2>> gpurun_out/r05z_bench.err
echo bench done
