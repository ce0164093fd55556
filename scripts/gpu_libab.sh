#!/bin/bash
# Bench A/B over diagnostic library builds: LIBS="build/libhge.so build/libhge_x1.so ..."
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-libab}
mkdir -p $OUT
for L in ${LIBS:-build/libhge.so}; do
  T=$(basename $L .so)
  HGE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > $OUT/b_$T.json 2> $OUT/b_$T.err || { tail -20 $OUT/b_$T.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/b_$T.json').read().strip().splitlines()[-1])
print('$T', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:30], list(d['kernels_ms_per_replay'].items())[:7])"
done
