#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-big}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --steps 3 --warmup 1 > $OUT/n64_1m.json 2> $OUT/n64_1m.err || { tail -5 $OUT/n64_1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 2000000 --steps 2 --warmup 1 > $OUT/n256_2m.json 2> $OUT/n256_2m.err || { tail -5 $OUT/n256_2m.err; exit 1; }
timeout -k 10 900 python -u bench.py --no-cpu-baseline --participants 256 --events 10000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_10m.json 2> $OUT/n256_10m.err || { tail -5 $OUT/n256_10m.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], d['ingest_host_ms'], round(sum(k.values()),2), list(k.items())[:14])
"; done
