#!/bin/bash
# Default bench (DSEC + workloads incl. hires1920 and e2e), as the driver runs it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06v
mkdir -p $OUT
S=$(date +%s); timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 3; }
echo "wall $(( $(date +%s) - S )) s"
python3 -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('dsec', d['value'], d['ms_per_step'])
for k,v in d['workloads'].items(): print(k, v.get('value'), v.get('ms_per_step'), v.get('wall_s'), v.get('error'))
"
