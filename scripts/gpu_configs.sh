#!/bin/bash
# the other configurations on the final build: 16/100k, 32/1M, 64/1M (config 3), 128/1M, and config 5 (Monte Carlo)
set -o pipefail
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
for NE in "16 100000" "32 1000000" "64 1000000" "128 1000000"; do
  set -- $NE
  timeout -k 10 300 python -u bench.py --participants $1 --events $2 --no-secondary --no-cpu-baseline --steps 5 --warmup 2 > $OUT/n$1_e$2.json 2> $OUT/n$1_e$2.err || { tail -20 $OUT/n$1_e$2.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/n$1_e$2.json').read().strip().splitlines()[-1])
print('$1/$2', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:90])"
done
timeout -k 10 400 python -u bench.py --workload mc --no-cpu-baseline --steps 3 --warmup 1 > $OUT/mc.json 2> $OUT/mc.err || { tail -20 $OUT/mc.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/mc.json').read().strip().splitlines()[-1])
print('mc', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:90])"
