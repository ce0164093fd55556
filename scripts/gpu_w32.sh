#!/bin/bash
# the int32 switch past 65,534 events per chain (forced low by HGE_CHAIN_LIMIT), then the store/wide suites
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-w32}
mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_store.py -k "uint16" > $OUT/pytest_w32.log 2>&1 || { echo "w32 tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_w32.log | head -30; tail -5 $OUT/pytest_w32.log; exit 1; }
tail -1 $OUT/pytest_w32.log
