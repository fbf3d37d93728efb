#!/bin/bash
# SQ / TA / TD / TCP / TCC passes over lookup_kernel alone (tools/kbench_lookup.hip, one shape and
# variant each), run via gpurun:   bash tools/gpu_lookup_pmc.sh <tag> <shape> ["<variant>"]
set -o pipefail
TAG=$1; SH=$2; V=${3:-prod launch_lookup}
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum"
P3="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_BUSY_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES"
OUT=gpurun_out/${TAG}_$SH
mkdir -p $OUT
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- ./tools/_build/kbench_lookup 3 $SH "$V" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 3; }
done
echo "$SH done"
