#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-wide}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_wide.log 2>&1; rc=$?
tail -25 $OUT/pytest_wide.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --k 64 --steps 3 --warmup 1 > $OUT/n64_1m.json 2>&1 || { tail -5 $OUT/n64_1m.json; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --k 256 --steps 2 --warmup 1 > $OUT/n256_1m.json 2>&1 || { tail -5 $OUT/n256_1m.json; exit 1; }
