#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-mc}
mkdir -p $OUT
HGE_WIDE=1 timeout -k 10 600 python -u bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline > $OUT/mc_wide.json 2> $OUT/mc_wide.err || { tail -20 $OUT/mc_wide.err; exit 1; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 600 python -u bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline --threads 16 > $OUT/mc_q16.json 2> $OUT/mc_q16.err || { tail -20 $OUT/mc_q16.err; exit 1; }
HGE_WIDE=1 timeout -k 10 300 python -u bench.py --participants 4 --events 1000 --k 4 --no-cpu-baseline > $OUT/n4_wide.json 2> $OUT/n4_wide.err || { tail -20 $OUT/n4_wide.err; exit 1; }
timeout -k 10 300 python -u bench.py --participants 4 --events 1000 --k 4 > $OUT/n4.json 2> $OUT/n4.err || { tail -20 $OUT/n4.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], d['parity'], round(sum(k.values()),3), list(k.items())[:5], d['cpu_baseline'])
"; done
