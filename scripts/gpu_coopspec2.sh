#!/bin/bash
# guess modes x walker counts at 64/1M, 128/1M, 256/2M; then 256/10M default
set -o pipefail
OUT=gpurun_out/${1:-coopspec}
mkdir -p $OUT
run() {  # n events walkers guess
HGE_WALK_DEBUG=1 HGE_COOP_WALKERS=$3 HGE_COOP_GUESS=$4 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 3 --warmup 1 --seed ${5:-1} > $OUT/n$1_w$3_g$4_s${5:-1}.json 2> $OUT/n$1_w$3_g$4_s${5:-1}.err || { tail -5 $OUT/n$1_w$3_g$4_s${5:-1}.err; exit 1; }
}
run 64 1000000 8 0 && run 64 1000000 8 1 && run 64 1000000 8 0 2 && run 64 1000000 8 1 2 && run 128 1000000 4 0 2 && run 128 1000000 4 1 2 && run 256 2000000 2 0 2 && run 256 2000000 2 1 2 || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --participants 256 --events 10000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_10m.json 2> $OUT/n256_10m.err || { tail -5 $OUT/n256_10m.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], list(k.items())[:3])
"; done
grep -h "coop walk" $OUT/*.err | sort | uniq -c | head -20
