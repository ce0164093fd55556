#!/bin/bash
# Per-kernel PMC diagnostics (one rocprofv3 pass per counter group, --kernel-trace only):
#   tcc: L2 hits / misses / memory-side read requests;  sq: wave-state and instruction mix.
# usage: scripts/gpu_pmc_diag.sh <tag> [bench args...]   (default 256 participants, 2M events)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-diag}
shift
ARGS=${*:---participants 256 --events 2000000}
mkdir -p $OUT
run() {
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $OUT/$1 -o pmc -- \
    python3 bench.py --no-cpu-baseline --no-secondary --steps 1 --warmup 0 --profile-steps 1 $ARGS > $OUT/$1.log 2>&1
}
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" || { echo "tcc pass failed"; tail -5 $OUT/tcc.log; exit 1; }
run sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
python3 scripts/pmc_diag_summary.py $OUT
