#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-seg}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for S in 64 32 16 8; do
  HGE_SEG=$S timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/seg$S.json 2>&1 || exit 1
  HGE_SEG=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/seg${S}_n256.json 2>&1 || exit 1
done
for f in $OUT/seg*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']; l=d['kernel_launches_per_replay']
sw=[a for a in k if 'la_sweep' in a][0]
print('$f', d['value'], d['ms_per_step'], sw, k[sw], l[sw], k.get('k_round_assign'))
"; done
