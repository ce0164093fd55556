#!/bin/bash
# Speculative wide walk: parity tests, then 64/1M, 128/1M and 256/2M at several walker counts.
set -o pipefail
OUT=gpurun_out/${1:-coopspec}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_coop_spec.py tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run() {  # n events walkers
HGE_WALK_DEBUG=1 HGE_COOP_WALKERS=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 3 --warmup 1 > $OUT/n$1_w$3.json 2> $OUT/n$1_w$3.err || { tail -5 $OUT/n$1_w$3.err; exit 1; }
}
run 64 1000000 4 && run 64 1000000 8 && run 128 1000000 2 && run 128 1000000 4 && run 256 2000000 0 && run 256 2000000 2 || exit 1
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], list(k.items())[:4])
"; done
grep -h "coop walk" $OUT/*.err | sort | uniq -c | head
