#!/bin/bash
# per-walker merge results of the speculative walk (HGE_WALK_DEBUG) at 16/100k
set -o pipefail
OUT=gpurun_out/${1:-walkdbg}
mkdir -p $OUT
for w in 16 32; do
  HGE_WALK_DEBUG=1 HGE_WALKERS=$w timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --profile-steps 1 > $OUT/w$w.json 2> $OUT/w$w.err || { tail -5 $OUT/w$w.err; exit 1; }
  grep "walk:" $OUT/w$w.err | head -2
done
