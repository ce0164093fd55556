#!/bin/bash
# round 3: revised rounds kernel parity + bench, stamps A/B, split emulation at 256/10M
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
bash scripts/gpu_quick.sh ${1:-r03e}_q || exit 1
LIBS="build/libhge_stamps.so build/old/libhge_stamps.so" bash scripts/gpu_stamps_ab.sh ${1:-r03e}_st || exit 2
timeout -k 10 500 python -u scripts/analysis/split_emulate.py 256 10000000 2 4 8 > $OUT/emulate.log 2>&1 || { tail -20 $OUT/emulate.log; exit 3; }
grep -E "unsplit|max part" $OUT/emulate.log
