#!/bin/bash
# per-section cycles of the wide rounds kernel (HGE_STAMPS, workgroup 0)
set -o pipefail
OUT=gpurun_out/${1:-coopstamps}
mkdir -p $OUT
for cfg in "64 1000000" "256 2000000"; do set -- $cfg
HGE_STAMPS=1 HGE_COOP_WALKERS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events $2 --steps 1 --warmup 0 > $OUT/n$1.json 2> $OUT/n$1.err || { tail -5 $OUT/n$1.err; exit 1; }
grep "hge stamps" $OUT/n$1.err | tail -1; grep -c "hge stamps" $OUT/n$1.err
done
