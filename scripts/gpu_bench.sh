#!/bin/bash
# bench lines: default workload (+ variants) and the Monte Carlo batch
set -o pipefail
OUT=gpurun_out/${1:-bench}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/default.json 2> $OUT/default.err || { tail -20 $OUT/default.err; exit 1; }
cat $OUT/default.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/wide16.json 2> $OUT/wide16.err || { tail -20 $OUT/wide16.err; exit 1; }
HGE_CHUNK=512 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/chunk512.json 2> $OUT/chunk512.err || { tail -20 $OUT/chunk512.err; exit 1; }
timeout -k 10 600 python -u bench.py --workload mc --steps 2 --warmup 1 > $OUT/mc.json 2> $OUT/mc.err || { tail -20 $OUT/mc.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['parity'], d['roofline']['kernel'], d['roofline']['frac'], list(d['kernels_ms_per_replay'].items())[:6])
"; done
