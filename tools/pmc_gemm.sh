#!/bin/bash
# Kernel trace + one PMC pass of the backward GEMM variants of tools/_build/kbench_gemm (run via
# gpurun).  Output under gpurun_out/pmc_gemm_<tag>/; summaries via tools/pmc_summary.py.
set -eo pipefail
TAG=${1:-run}
OUT=gpurun_out/pmc_gemm_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "dF1 (rows) bf16x6 256x256 pipelined" "dF2 (cols) bf16x6 256x256 pipelined" \
         "dF1 (rows) DMA mix splits plan, 256x256 pipelined" "dF2 (cols) DMA mix splits plan, 256x256 pipelined"; do
    d="$OUT/$(echo "$v" | tr -c 'A-Za-z0-9' '_')"
    mkdir -p "$d"
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$d/trace" -o run --output-format csv -- ./tools/_build/kbench_gemm 5 "$v" > "$d/kbench.txt" 2> "$d/trace.err"
    timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -d "$d/pmc1" -o run --output-format csv -- ./tools/_build/kbench_gemm 2 "$v" > /dev/null 2> "$d/pmc1.err"
    python3 tools/pmc_summary.py "$d" --json "$d/pmc.json" > "$d/summary.txt"
    rm -f "$d"/*/*/*counter_collection.csv "$d"/*/*/*kernel_trace.csv "$d"/*/*counter_collection.csv "$d"/*/*kernel_trace.csv
    echo "== $v"; grep -E "split_gemm|splitk|avg_us|MFMA|GRBM|SQ_BUSY" "$d/summary.txt"
done
