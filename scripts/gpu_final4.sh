#!/bin/bash
# Full GPU pass: every parity test, smoke, headline bench + rocprof stats (csv), 64/1M, 128/1M, 256/10M.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final4}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { grep -v "^    @" $OUT/prof.log | tail -5; exit 1; }
timeout -k 10 300 python -u bench.py --participants 64 --events 1000000 --steps 3 --warmup 1 --cpu-sample-events 20000 > $OUT/n64_1m.json 2> $OUT/n64_1m.err || { tail -5 $OUT/n64_1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 128 --events 1000000 --steps 3 --warmup 1 > $OUT/n128_1m.json 2> $OUT/n128_1m.err || { tail -5 $OUT/n128_1m.err; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline --participants 256 --events 10000000 --steps 2 --warmup 1 --profile-steps 1 > $OUT/n256_10m.json 2> $OUT/n256_10m.err || { tail -5 $OUT/n256_10m.err; exit 1; }
for f in $OUT/*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', round(d['value']/1e6,2), d['ms_per_step'], d.get('parity'), d['roofline']['kernel'], d['roofline']['frac'], list(k.items())[:3])
"; done
