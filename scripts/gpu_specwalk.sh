#!/bin/bash
# speculative frontier walk: its parity tests, then the full GPU suite, then
# bench lines with and without it
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-specwalk}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec_walk.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_spec.log 2>&1 || { echo "spec tests failed"; tail -40 $OUT/pytest_spec.log; exit 1; }
tail -3 $OUT/pytest_spec.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
HGE_WALKERS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_seq.json 2> $OUT/bench_seq.err || { echo "bench seq failed"; tail -30 $OUT/bench_seq.err; exit 1; }
for f in $OUT/bench*.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$f', d['value'], d['ms_per_step'], d['parity'], d['roofline']['kernel'], d['roofline']['frac'], list(k.items())[:8])
"; done
