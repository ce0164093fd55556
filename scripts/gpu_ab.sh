#!/bin/bash
# A/B runs: parity under both lastAncestors kernels, bench lines, direct-rounds section stamps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_wide.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/pt_block.log 2>&1 || { tail -30 $OUT/pt_block.log; exit 1; }
tail -1 $OUT/pt_block.log
HGE_LW_KERNEL=wave timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/pt_wave.log 2>&1 || { tail -30 $OUT/pt_wave.log; exit 1; }
tail -1 $OUT/pt_wave.log
for K in block wave; do
  HGE_LW_KERNEL=$K timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $OUT/b_$K.json 2> $OUT/b_$K.err || { tail -20 $OUT/b_$K.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/b_$K.json').read().strip().splitlines()[-1])
print('$K', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:40], list(d['kernels_ms_per_replay'].items())[:7])"
done
HGE_LIB=build/libhge_stamps.so HGE_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --participants 256 --events 2000000 --steps 1 --warmup 0 --ramp-s 0 --profile-steps 1 > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
grep "hge stamps" $OUT/st.err | tail -2
python -c "
import json
d=json.loads(open('$OUT/st.json').read().strip().splitlines()[-1])
print('stamps run', d['rounds'], list(d['kernels_ms_per_replay'].items())[:3])"
