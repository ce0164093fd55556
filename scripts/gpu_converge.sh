#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-conv}
mkdir -p $OUT
timeout -k 10 200 python -u scripts/analysis/split_converge.py 64 40000 2 4 > $OUT/c64.log 2>&1 || { tail -20 $OUT/c64.log; exit 1; }
cat $OUT/c64.log
timeout -k 10 400 python -u scripts/analysis/split_converge.py 256 10000000 2 4 8 > $OUT/c256.log 2>&1 || { tail -20 $OUT/c256.log; exit 1; }
cat $OUT/c256.log
