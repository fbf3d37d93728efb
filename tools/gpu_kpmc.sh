#!/bin/bash
# SQ / TA / TD / TCP / TCC passes over one kernel-bench variant each, run via gpurun:
#   bash tools/gpu_kpmc.sh <tag> <binary> "<variant>" ["<variant>" ...]
set -o pipefail
TAG=$1; BIN=$2; shift 2
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum"
P3="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_BUSY_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
v=0
for V in "$@"; do
  v=$((v+1))
  OUT=gpurun_out/${TAG}_v$v
  mkdir -p $OUT
  echo "$V" > $OUT/variant.txt
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- $BIN 3 "$V" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 3; }
  done
  echo "variant $v done"
done
