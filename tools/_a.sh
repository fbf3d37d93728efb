set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/kbench_aux.py > gpurun_out/aux.json 2> gpurun_out/aux.err; rc=$?; cat gpurun_out/aux.json; tail -3 gpurun_out/aux.err; exit $rc
