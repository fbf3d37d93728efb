#!/bin/bash
# Fold variants A/B (interleaved) + LDS / VALU PMC of each:  bash tools/gpu_r06e.sh <tag> <binary>...
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
V="SEP full T=12, no maxima (bf16x6)"
for r in 1 2; do
  for b in "$@"; do
    echo "== $b round $r" >> $OUT/ab.txt
    timeout -k 10 120 ./tools/_build/$b 8 >> $OUT/ab.txt 2>&1 || { echo "$b failed"; exit 3; }
  done
done
echo ab done
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
for b in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_$b -o run --output-format csv -- ./tools/_build/$b 3 "$V" > $OUT/pmc_$b.log 2>&1 || { echo "pmc $b failed"; exit 4; }
done
echo pmc done
