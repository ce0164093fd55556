#!/bin/bash
# Section stamps of the direct rounds kernel (workgroup 0) at 256/2M (STAMP_EVENTS=10000000: 256/10M), from the stamps build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-stamps}
mkdir -p $OUT
HGE_LIB=build/libhge_stamps.so HGE_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --participants 256 --events ${STAMP_EVENTS:-2000000} --steps 1 --warmup 0 --ramp-s 0 --profile-steps 1 > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep "hge stamps" $OUT/st.err | tail -3
python -c "
import json
d=json.loads(open('$OUT/st.json').read().strip().splitlines()[-1])
print('rounds', d['rounds'], d['ms_per_step'], list(d['kernels_ms_per_replay'].items())[:3])"
