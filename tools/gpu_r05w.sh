set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --workload train > gpurun_out/r05w_bench_train.json 2> gpurun_out/r05w_bench_train.err
ERAFT_AMD_EXACT_FOLD=1 timeout -k 10 300 python3 -u bench.py --workload train --no-cpu-baseline > gpurun_out/r05w_bench_train_exactfold.json 2> gpurun_out/r05w_bench_train_exactfold.err
timeout -k 10 300 python3 -u bench.py --workload train --no-cpu-baseline > gpurun_out/r05w_bench_train2.json 2>> gpurun_out/r05w_bench_train.err
echo done
