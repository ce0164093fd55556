#!/bin/bash
# parity + bench, then the sharded split emulated part by part on one GPU (256/10M)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-emu}
mkdir -p $OUT
bash scripts/gpu_quick.sh ${1:-emu}_q || exit 1
timeout -k 10 600 python -u scripts/analysis/split_emulate.py 256 10000000 2 4 8 > $OUT/emulate.log 2>&1 || { tail -20 $OUT/emulate.log; exit 3; }
grep -E "unsplit|max part" $OUT/emulate.log
