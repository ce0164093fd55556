#!/bin/bash
# round 3 final: full GPU suite, smoke, bench (secondary lines and CPU baseline), rocprofv3 kernel stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03f}
mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['ms_per_step'], d['parity'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'])
print(list(d['kernels_ms_per_replay'].items())[:8])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $OUT/prof.log 2>&1
echo "rocprofv3 rc=$?"
