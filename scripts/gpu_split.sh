#!/bin/bash
# the sharded split tests alone (verbose), then the rest of the r03d pass
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-split}
mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 240 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_split.py -k sharded > $OUT/pytest_sharded.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_sharded.log | tail -12
exit $rc
