#!/bin/bash
# fame window width (HGE_SPEC) sweep on the default bench
set -o pipefail
OUT=gpurun_out/${1:-spec}
mkdir -p $OUT
for S in 2 3 4 6; do
  HGE_SPEC=$S timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/spec$S.json 2>&1 || exit 1
done
for f in $OUT/spec*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], d['parity'], k.get('k_fame_decide<1>'), k.get('k_fame_timeline_g<16>'), k.get('k_lcr_scan'))
"; done
