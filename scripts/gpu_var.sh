#!/bin/bash
# run-to-run spread of the default bench line (no tests)
set -o pipefail
OUT=gpurun_out/${1:-var}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/b$i.json 2>&1 || exit 1
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 50 --warmup 10 > $OUT/s$i.json 2>&1 || exit 1
done
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'])
"; done
