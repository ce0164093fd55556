#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final2}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 128 --events 1000000 --steps 3 --warmup 1 > $OUT/n128_1m.json 2> $OUT/n128_1m.err || { tail -5 $OUT/n128_1m.err; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline --participants 256 --events 10000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_10m.json 2> $OUT/n256_10m.err || { tail -5 $OUT/n256_10m.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof64 -o run -- python3 bench.py --no-cpu-baseline --participants 64 --events 1000000 --steps 2 --warmup 1 > $OUT/prof64.log 2>&1 || { grep -v "^    @" $OUT/prof64.log | tail -5; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], list(k.items())[:4])
"; done
find $OUT/prof64 -name "*stats*"
