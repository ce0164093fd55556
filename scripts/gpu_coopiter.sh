#!/bin/bash
# wide-walk iteration: wide parity tests, section stamps, 64/1M + 128/1M + 256/2M benches
set -o pipefail
OUT=gpurun_out/${1:-coopiter}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_coop_spec.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in "64 1000000" "256 2000000"; do set -- $cfg
HGE_STAMPS=1 HGE_COOP_WALKERS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 1 --warmup 0 > $OUT/st$1.json 2> $OUT/st$1.err || { tail -5 $OUT/st$1.err; exit 1; }
grep "hge stamps" $OUT/st$1.err | tail -1
done
for cfg in "64 1000000" "128 1000000" "256 2000000"; do set -- $cfg
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 3 --warmup 1 > $OUT/n$1.json 2> $OUT/n$1.err || { tail -5 $OUT/n$1.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/n$1.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('n$1', round(d['value']/1e6,2), d['ms_per_step'], list(k.items())[:3])
"
done
