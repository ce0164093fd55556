#!/bin/bash
# full GPU suite, then the online per-call probe (host round trips, p50/p99)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 1000 $PYT tests -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -30; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u scripts/online_probe.py > $OUT/online.json 2> $OUT/online.err || { tail -20 $OUT/online.err; exit 2; }
cat $OUT/online.json
