#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench (1 step), then the PMC traffic passes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $OUT/prof.log 2>&1
echo "rocprofv3 rc=$?"
tail -1 $OUT/prof.log | cut -c1-300
bash scripts/gpu_pmc.sh ${1:-prof}_pmc
