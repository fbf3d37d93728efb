#!/bin/bash
# PMC passes over split_gemm_f32_kernel alone (tools/kbench_gemm.hip, one variant), run via gpurun:
#   bash tools/gpu_gemm_pmc.sh "<variant name>" <tag>
set -o pipefail
V=${1:-dF1 (rows) reg splits plan}
OUT=gpurun_out/gemm_pmc_${2:-a}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- ./tools/_build/kbench_gemm 3 "$V" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 3; }
done
echo done
