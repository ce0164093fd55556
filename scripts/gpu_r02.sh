#!/bin/bash
# Round-2 GPU pass: parity tests, smoke, default bench (256/10M), rocprofv3 kernel stats.
# usage: scripts/gpu_r02.sh <tag> [tests|bench|prof|segv|all] [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02}
WHAT=${2:-all}
mkdir -p $OUT
if [[ $WHAT == all || $WHAT == tests ]]; then
  K=${3:+-k "$3"}
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread $K > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "PASS|FAIL|ERROR" $OUT/pytest_gpu.log | tail -5; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['ms_per_step'], d['parity'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'])
print(json.dumps(d.get('secondary')))
print(list(d['kernels_ms_per_replay'].items())[:8])"
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  HGE_DUMP_MAPS=$OUT/maps.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $OUT/prof.log 2>&1
  echo "rocprofv3 (plain launches) rc=$?"
  grep -v "^W2\|^E2" $OUT/prof.log | tail -3
fi
if [[ $WHAT == segv ]]; then
  # exit-time SIGSEGV under rocprofv3: cooperative launch vs plain launch, same bench
  for mode in 0 1; do
    HGE_COOP_LAUNCH=$mode HGE_DUMP_MAPS=$OUT/maps_coop$mode.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_coop$mode -o run -- python3 bench.py --no-cpu-baseline --no-secondary --participants 64 --events 200000 --steps 2 --warmup 1 > $OUT/prof_coop$mode.log 2>&1
    echo "HGE_COOP_LAUNCH=$mode rocprofv3 rc=$?"
  done
fi
