#!/bin/bash
# wide configs after a change: parity tests, 256/1M and 256/10M lines
set -o pipefail
OUT=gpurun_out/${1:-wide2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --steps 2 --warmup 1 > $OUT/n256_1m.json 2> $OUT/n256_1m.err || { tail -5 $OUT/n256_1m.err; exit 1; }
timeout -k 10 900 python -u bench.py --no-cpu-baseline --participants 256 --events 10000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_10m.json 2> $OUT/n256_10m.err || { tail -5 $OUT/n256_10m.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], list(k.items())[:10])
"; done
