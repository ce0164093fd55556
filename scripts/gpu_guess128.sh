#!/bin/bash
# guess type for the 2 x 1024-thread walkers at 128/1M over seeds 1-3
set -o pipefail
OUT=gpurun_out/${1:-guess128}
mkdir -p $OUT
for s in 1 2 3; do for g in 1 2; do
HGE_COOP_GUESS=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 128 --events 1000000 --steps 2 --warmup 1 --seed $s > $OUT/g${g}_s$s.json 2> $OUT/g${g}_s$s.err || { tail -5 $OUT/g${g}_s$s.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/g${g}_s$s.json').read().strip().splitlines()[-1])
print('g$g s$s', round(d['value']/1e6,2), d['kernels_ms_per_replay'].get('k_rounds_coop_spec'))
"
done; done
