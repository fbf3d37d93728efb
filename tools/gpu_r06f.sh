#!/bin/bash
# Fold: backward parity tests, A/B (HEAD vs working tree kbench_bwd), PMC of the lean variant.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06f
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "backward or bwd or config4 or fold or staged or autograd" > $OUT/tests.txt 2>&1 || { echo tests failed; tail -30 $OUT/tests.txt; exit 2; }
tail -2 $OUT/tests.txt
for r in 1 2; do
  for b in kbench_bwd_old kbench_bwd; do
    echo "== $b round $r" >> $OUT/ab.txt
    timeout -k 10 150 ./tools/_build/$b 8 >> $OUT/ab.txt 2>&1 || { echo "$b failed"; exit 3; }
  done
done
echo ab done
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/pmc_lean -o run --output-format csv -- ./tools/_build/kbench_bwd 3 "SEP LEAN full T=12, no maxima (bf16x6)" > $OUT/pmc_lean.log 2>&1 || { echo "pmc failed"; exit 4; }
echo pmc done
