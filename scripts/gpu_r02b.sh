#!/bin/bash
# Full GPU parity suite + smoke, then default bench vs an env A/B (ABENV).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for AB in "X=0" ${ABENV}; do
  env $AB timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > $OUT/b_$AB.json 2> $OUT/b_$AB.err || { tail -20 $OUT/b_$AB.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/b_$AB.json').read().strip().splitlines()[-1])
print('$AB', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:40], list(d['kernels_ms_per_replay'].items())[:6])"
done
