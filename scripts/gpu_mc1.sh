#!/bin/bash
# configs 1 and 5: 4/1k gossip and the Monte Carlo batch (1024 x N=32, forkers)
set -o pipefail
OUT=gpurun_out/${1:-mc1}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --participants 4 --events 1000 --k 4 --steps 20 --warmup 5 > $OUT/n4_1k.json 2> $OUT/n4_1k.err || { tail -5 $OUT/n4_1k.err; exit 1; }
timeout -k 10 600 python -u bench.py --workload mc --steps 2 --warmup 1 > $OUT/mc.json 2> $OUT/mc.err || { tail -5 $OUT/mc.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', round(d['value']/1e6,2), d['ms_per_step'], d.get('parity'), (d.get('cpu_baseline') or {}).get('value'))
"; done
