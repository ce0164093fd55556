#!/bin/bash
# fame window width on the wide configs
set -o pipefail
OUT=gpurun_out/${1:-spec2}
mkdir -p $OUT
for S in 3 6; do
  HGE_SPEC=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n64_spec$S.json 2>&1 || exit 1
  HGE_SPEC=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_spec$S.json 2>&1 || exit 1
done
for f in $OUT/n*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
fd=[v for a,v in k.items() if 'fame_decide' in a]
print('$f', d['value'], d['ms_per_step'], fd, k.get('k_lcr_scan'), d['kernel_launches_per_replay'].get('k_lcr_scan'))
"; done
