#!/bin/bash
# parity of the current build on the wide goldens and store tests, then a bench A/B against build/libhge_base.so
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-abq}
mkdir -p $OUT
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_golden.py tests/test_gpu_wide.py tests/test_gpu_store.py > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAIL|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
LIBS="build/libhge.so build/libhge_base.so build/libhge.so build/libhge_base.so" bash scripts/gpu_libab.sh $1
