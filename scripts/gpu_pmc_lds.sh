#!/bin/bash
# LDS / VALU activity of the rounds kernel at 256/2M (one PMC pass, 8 SQ counters)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_lds}
mkdir -p $OUT
timeout -k 10 300 python3 scripts/pmc_sq.py $OUT --counters SQ_WAVES,SQ_WAVE_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VALU -- --no-secondary --participants 256 --events 2000000 --steps 1 --warmup 0 > $OUT/lds.txt 2> $OUT/lds.err || { tail -30 $OUT/lds.err; exit 1; }
head -12 $OUT/lds.txt
