#!/bin/bash
# walker-count sweep of the speculative frontier walk at 16/100k and 32-wide
set -o pipefail
OUT=gpurun_out/${1:-walkers}
mkdir -p $OUT
for w in 8 12 16 24 32 48; do
  HGE_WALKERS=$w timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/w$w.json 2> $OUT/w$w.err || { tail -5 $OUT/w$w.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/w$w.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('w=$w', d['value'], d['ms_per_step'], [(n,v) for n,v in k.items() if 'walk' in n])
"
done
