#!/bin/bash
# GPU pass (round 3): parity tests, smoke, default bench (256/10M), rocprofv3 kernel stats.
# usage: scripts/gpu_r02.sh <tag> [tests|bench|prof|segv|all] [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03}
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
if [[ $WHAT == quick ]]; then
  # wide-path parity + headline numbers without the CPU legs
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or coop or fullsize or wide or store or gpu_parity or split or reference" > $OUT/pytest_quick.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_quick.log; exit 1; }
  tail -1 $OUT/pytest_quick.log
  for cfg in "256 10000000" "64 1000000" "128 1000000"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --participants $1 --events $2 --steps 3 --warmup 1 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { tail -20 $OUT/b_$1_$2.err; exit 1; }
    python -c "
import json
d=json.loads(open('$OUT/b_$1_$2.json').read().strip().splitlines()[-1])
print('$1/$2', round(d['value']/1e6,2), 'Mev/s', d['ms_per_step'], 'ms', d['parity'], list(d['kernels_ms_per_replay'].items())[:6])"
  done
fi
if [[ $WHAT == stamps ]]; then
  # section cycles of the direct rounds step (workgroup 0), and median / rounds A/B
  HGE_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --participants 256 --events 2000000 --steps 1 --warmup 0 --ramp-s 0 --profile-steps 1 > $OUT/st.json 2> $OUT/st.err || { tail -20 $OUT/st.err; exit 1; }
  grep "hge stamps" $OUT/st.err | tail -2
  for env in ${ABENVS:-HGE_SWEEP_SKIP=0 HGE_MEDIAN_ORDER=chain X=1}; do
    env $env timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --participants 256 --events 2000000 --steps 3 --warmup 1 > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
    python -c "
import json
d=json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
print('$env', round(d['value']/1e6,2), d['ms_per_step'], list(d['kernels_ms_per_replay'].items())[:5])"
  done
fi
if [[ $WHAT == all || $WHAT == converge ]]; then
  # how far split walkers must overlap
  timeout -k 10 300 python -u scripts/analysis/split_converge.py 256 10000000 2 4 8 > $OUT/converge.log 2>&1 || { tail -20 $OUT/converge.log; exit 1; }
  tail -3 $OUT/converge.log
fi
