set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload e2e --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/be2e_g.json 2> gpurun_out/be2e_g.err; cat gpurun_out/be2e_g.json; tail -3 gpurun_out/be2e_g.err
