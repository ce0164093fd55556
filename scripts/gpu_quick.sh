#!/bin/bash
# quick bench lines over the main configs (no tests)
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/n16.json 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n64.json 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256.json 2>&1 || exit 1
for f in $OUT/n*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['hbm_kernels'])
"; done
