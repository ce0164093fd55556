#!/bin/bash
# Speculative wide walk: parity tests, then 64/1M and 128/1M with and without walkers.
set -o pipefail
OUT=gpurun_out/${1:-coopspec}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_coop_spec.py tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for nw in 0 4; do
HGE_WALK_DEBUG=1 HGE_COOP_WALKERS=$nw timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --steps 3 --warmup 1 > $OUT/n64_w$nw.json 2> $OUT/n64_w$nw.err || { tail -5 $OUT/n64_w$nw.err; exit 1; }
done
for nw in 0 2; do
HGE_WALK_DEBUG=1 HGE_COOP_WALKERS=$nw timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 128 --events 1000000 --steps 3 --warmup 1 > $OUT/n128_w$nw.json 2> $OUT/n128_w$nw.err || { tail -5 $OUT/n128_w$nw.err; exit 1; }
done
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], d['parity'], list(k.items())[:6])
"; done
grep -h "coop walk" $OUT/*.err | sort | uniq -c | head
