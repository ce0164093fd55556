#!/bin/bash
# Section stamps of the direct rounds kernel (workgroup 0) at 256/2M for several
# stamps builds: LIBS="build/libhge_stamps.so build/old/libhge_stamps.so"
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-stampsab}
mkdir -p $OUT
for L in ${LIBS:-build/libhge_stamps.so}; do
  T=$(echo $L | tr '/' '_')
  HGE_LIB=$L HGE_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --participants 256 --events 2000000 --steps 1 --warmup 0 --ramp-s 0 --profile-steps 1 > $OUT/st_$T.json 2> $OUT/st_$T.err || { tail -20 $OUT/st_$T.err; exit 1; }
  echo "$L"; grep "hge stamps" $OUT/st_$T.err | tail -1
  python -c "
import json
d=json.loads(open('$OUT/st_$T.json').read().strip().splitlines()[-1])
print('rounds', d['rounds'], d['ms_per_step'], list(d['kernels_ms_per_replay'].items())[:3])"
done
