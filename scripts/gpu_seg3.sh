#!/bin/bash
# sweep segment length at 16/100k (HGE_SEG)
set -o pipefail
OUT=gpurun_out/${1:-seg3}
mkdir -p $OUT
for S in 16 32 64; do
  HGE_SEG=$S timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/seg$S.json 2>&1 || exit 1
done
for f in $OUT/seg*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']; l=d['kernel_launches_per_replay']
sw=[a for a in k if 'la_sweep' in a][0]
print('$f', d['value'], d['ms_per_step'], k[sw], l[sw])
"; done
