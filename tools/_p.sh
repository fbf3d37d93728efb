set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_train
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train/trace -o run --output-format csv -- python3 bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_train/b.json 2> gpurun_out/prof_train/err.txt
