#!/bin/bash
# every BASELINE config on one GPU: 4/1k (with CPU baseline), 16/100k (default line),
# 64/1M, 256/1M, 256/2M, 256/10M, and the Monte Carlo batch (1024 x N=32 x 10k)
set -o pipefail
OUT=gpurun_out/${1:-all}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --participants 4 --events 1000 --k 4 > $OUT/n4_1k.json 2> $OUT/n4_1k.err || { tail -5 $OUT/n4_1k.err; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/n16_100k.json 2> $OUT/n16_100k.err || { tail -5 $OUT/n16_100k.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --steps 3 --warmup 1 > $OUT/n64_1m.json 2> $OUT/n64_1m.err || { tail -5 $OUT/n64_1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --steps 2 --warmup 1 > $OUT/n256_1m.json 2> $OUT/n256_1m.err || { tail -5 $OUT/n256_1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 2000000 --steps 2 --warmup 1 > $OUT/n256_2m.json 2> $OUT/n256_2m.err || { tail -5 $OUT/n256_2m.err; exit 1; }
timeout -k 10 900 python -u bench.py --no-cpu-baseline --participants 256 --events 10000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_10m.json 2> $OUT/n256_10m.err || { tail -5 $OUT/n256_10m.err; exit 1; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 600 python -u bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline --threads 16 > $OUT/mc.json 2> $OUT/mc.err || { tail -20 $OUT/mc.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], d['parity'], d['roofline']['kernel'], d['roofline']['frac'], list(k.items())[:6])
"; done
