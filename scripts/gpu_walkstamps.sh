#!/bin/bash
OUT=gpurun_out/${1:-ws}
mkdir -p $OUT
HGE_STAMPS=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --profile-steps 1 > $OUT/n16.json 2> $OUT/n16.err || exit 1
grep stamps $OUT/n16.err | head -3
