#!/bin/bash
# PMC passes over lookup_bwd_fold_kernel alone (tools/kbench_bwd.hip, one variant), run via gpurun:
#   bash tools/gpu_fold_pmc.sh "<variant name>"
set -o pipefail
V=${1:-full T=12}
OUT=gpurun_out/fold_pmc
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD"
P3="SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- ./tools/_build/kbench_bwd 3 "$V" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 3; }
done
echo done
