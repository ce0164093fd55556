#!/bin/bash
# checker-thread / poll-pause sweep of the speculative walk at 16/100k
set -o pipefail
OUT=gpurun_out/${1:-walkchk}
mkdir -p $OUT
for cfg in 448,2 192,2 64,2 64,16 192,8 448,8 896,2; do
 for w in 16 32; do
  HGE_WALK_CHK=$cfg HGE_WALKERS=$w timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/c${cfg}_w$w.json 2> $OUT/c${cfg}_w$w.err || { tail -5 $OUT/c${cfg}_w$w.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/c${cfg}_w$w.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('chk=$cfg w=$w', d['value'], d['ms_per_step'], [(n,v) for n,v in k.items() if 'walk' in n])
"
 done
done
