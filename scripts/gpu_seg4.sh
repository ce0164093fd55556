#!/bin/bash
# repeated A/B of the sweep segment length at 16/100k
set -o pipefail
OUT=gpurun_out/${1:-seg4}
mkdir -p $OUT
for i in 1 2 3; do
  for S in 16 64; do
    HGE_SEG=$S timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/seg${S}_$i.json 2>&1 || exit 1
  done
done
for f in $OUT/seg*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['replay_ms']['gpu'])
"; done
