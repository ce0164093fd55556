#!/bin/bash
# sequential wide walk (HGE_COOP_WALKERS=0) vs default walkers at 64/1M, 128/1M, 256/2M
set -o pipefail
OUT=gpurun_out/${1:-coopseq}
mkdir -p $OUT
for cfg in "64 1000000" "128 1000000" "256 2000000"; do set -- $cfg
HGE_COOP_WALKERS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 3 --warmup 1 > $OUT/seq$1.json 2> $OUT/seq$1.err || { tail -5 $OUT/seq$1.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/seq$1.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('seq n$1', round(d['value']/1e6,2), d['ms_per_step'], list(k.items())[:2])
"
done
