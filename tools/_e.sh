set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_e2e
timeout -k 10 300 python bench.py --workload e2e --steps 10 --warmup 3 --cpu-seconds 10 > gpurun_out/be2e.json 2> gpurun_out/be2e.err && cat gpurun_out/be2e.json && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e/trace -o run --output-format csv -- python3 bench.py --workload e2e --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_e2e/b.json 2> gpurun_out/prof_e2e/err.txt
