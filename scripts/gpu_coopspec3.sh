#!/bin/bash
# alternating guesses: 64/1M and 128/1M over seeds 1-3
set -o pipefail
OUT=gpurun_out/${1:-coopspec}
mkdir -p $OUT
run() {  # n events walkers guess seed
HGE_WALK_DEBUG=1 HGE_COOP_WALKERS=$3 HGE_COOP_GUESS=$4 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 2 --warmup 1 --seed $5 > $OUT/n$1_w$3_g$4_s$5.json 2> $OUT/n$1_w$3_g$4_s$5.err || { tail -5 $OUT/n$1_w$3_g$4_s$5.err; exit 1; }
}
for s in 1 2 3; do run 64 1000000 8 2 $s && run 128 1000000 4 2 $s && run 128 1000000 4 0 $s && run 128 1000000 0 0 $s || exit 1; done
run 64 1000000 8 0 3 && run 64 1000000 8 1 3 && run 64 1000000 0 0 3 || exit 1
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', round(d['value']/1e6,1), d['ms_per_step'], list(k.items())[:1])
"; done
