#!/bin/bash
# per-walker cycles of the speculative walk under different checker settings (w=32, 16/100k)
set -o pipefail
OUT=gpurun_out/${1:-walkdbg2}
mkdir -p $OUT
for cfg in ${CFGS:-448,2 192,2}; do
  HGE_WALK_CHK=$cfg HGE_WALK_DEBUG=1 HGE_WALKERS=32 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --profile-steps 1 > $OUT/c$cfg.json 2> $OUT/c$cfg.err || { tail -5 $OUT/c$cfg.err; exit 1; }
  echo "cfg $cfg"; grep "walk:" $OUT/c$cfg.err | tail -1
done
