set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_aux
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aux/trace -o run --output-format csv -- python3 tools/kbench_aux.py > gpurun_out/prof_aux/out.json 2> gpurun_out/prof_aux/err.txt
