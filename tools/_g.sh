set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?; tail -25 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
