# PMC passes over tools/_build/kbench_build (run via gpurun):  bash tools/pmc_kbench.sh <shape> <variant-substring>
set -o pipefail
SH=${1:-dsec}; VAR=${2:-"x3 mfma persist"}
OUT=gpurun_out/pk
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
K="./tools/_build/kbench_build 3 $SH"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE" \
         "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- $K "$VAR" > /dev/null 2>$OUT/p$i.err || echo "pass $i failed"
done
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- $K "$VAR" > $OUT/kb.txt 2>$OUT/tr.err || exit 5
echo done
