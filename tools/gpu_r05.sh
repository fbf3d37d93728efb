#!/bin/bash
# Round-5 measurement pass (run via gpurun): the bench line of every workload at HEAD, the
# launcher-less 2-rank rehearsal of the row-sharded 1280x960 path (gloo, both ranks on the one
# GPU), and a kernel trace of the DSEC and 1280x960 benches.
#   bash tools/gpu_r05.sh <tag>
# BENCH=0 skips the bench lines and the rehearsal; PROF="w1 w2" picks the profiled workloads.
set -eo pipefail
TAG=${1:-r05}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${BENCH:-1}" = 1 ]; then
for w in dsec train mvsec mvsec_crop hires1280 hires1920; do
  timeout -k 10 240 python3 -u bench.py --workload $w > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err
  echo "$w done"
done
ERAFT_AMD_DIST_BACKEND=gloo timeout -k 10 300 python3 -u bench.py --gpus 2 --workload hires1280 --sharded --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_hires1280_sharded2_gloo.json 2> gpurun_out/${TAG}_bench_hires1280_sharded2_gloo.err
echo "sharded gloo done"
fi
for w in ${PROF:-dsec hires1280}; do
  OUT=gpurun_out/prof_${TAG}_$w
  mkdir -p "$OUT"
  ARGS="--workload $w --no-cpu-baseline --steps 20 --warmup 5"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc2" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc2.err"
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3" -o run --output-format csv -- python3 bench.py $ARGS > /dev/null 2> "$OUT/pmc3.err"
  python3 tools/pmc_summary.py "$OUT" --json "$OUT/pmc.json" > "$OUT/summary.txt"
  echo "prof $w done"
done
