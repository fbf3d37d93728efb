#!/bin/bash
# A/B pass (run via gpurun): the division check, the GPU test suite, then old and new kernel
# benches interleaved.   bash tools/gpu_ab.sh <tag> [pytest -k expr]
set -eo pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/_build/kbench_div ]; then
  timeout -k 10 300 ./tools/_build/kbench_div 4096 > gpurun_out/${TAG}_div.txt 2>&1
  echo "div done"
fi
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "$2" > gpurun_out/${TAG}_tests.txt 2>&1
else
  timeout -k 10 700 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/${TAG}_tests.txt 2>&1
fi
echo "tests done"
for k in bwd lookup; do
  for v in base new base new; do
    b=tools/_build/kbench_$k; [ $v = base ] && b=${b}_base
    [ -x $b ] || continue
    echo "== $v" >> gpurun_out/${TAG}_kbench_$k.txt
    timeout -k 10 180 $b 10 >> gpurun_out/${TAG}_kbench_$k.txt 2>&1
  done
  echo "kbench $k done"
done
