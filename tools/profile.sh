#!/bin/bash
# Kernel-trace + PMC passes of bench.py on the GPU box (run via gpurun).  Output under
# gpurun_out/prof_<tag>/ ; copy the summaries worth keeping into profiles/.
#   tools/profile.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-run}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# PROG=tools/time_conv_bwd.py tools/profile.sh <tag> [args]: profile another script instead
PROG=${PROG:-bench.py}
if [ "$PROG" = bench.py ]; then ARGS="--no-cpu-baseline --steps 50 --warmup 10 $*"; else ARGS="$*"; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $PROG $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
# PMC in separate passes (never combined with --sys-trace / runtime traces)
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -k 10 240 rocprofv3 --pmc $P1 -d "$OUT/pmc1" -o run --output-format csv -- python3 $PROG $ARGS > /dev/null 2> "$OUT/pmc1.err"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2" -o run --output-format csv -- python3 $PROG $ARGS > /dev/null 2> "$OUT/pmc2.err"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3" -o run --output-format csv -- python3 $PROG $ARGS > /dev/null 2> "$OUT/pmc3.err"
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$OUT/pmc4" -o run --output-format csv -- python3 $PROG $ARGS > /dev/null 2> "$OUT/pmc4.err" || true
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA -d "$OUT/pmc5" -o run --output-format csv -- python3 $PROG $ARGS > /dev/null 2> "$OUT/pmc5.err" || true
python3 tools/pmc_summary.py "$OUT" --json "$OUT/pmc.json" > "$OUT/summary.txt"
echo done
