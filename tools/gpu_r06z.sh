#!/bin/bash
# bf16x6 backward GEMMs with s_setprio(1) around the MFMA region: A/B vs HEAD.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06z
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_bwd_bf16.py 20 > $OUT/ab.txt 2>&1 || { echo ab failed; tail -30 $OUT/ab.txt; exit 2; }
grep -v amdgpu.ids $OUT/ab.txt
