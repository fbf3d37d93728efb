set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for f in 1 0; do
ERAFT_AMD_FUSE_CONV=$f timeout -k 10 200 python bench.py --workload e2e --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/e2e_f$f.json 2>/dev/null || exit 5
python3 -c "import json; d=json.load(open('gpurun_out/e2e_f$f.json')); print('fuse=$f', d['value'], d['ms_per_step'])"
done; done
