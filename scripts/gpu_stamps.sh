#!/bin/bash
OUT=gpurun_out/${1:-stamps}
mkdir -p $OUT
HGE_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --k 64 --steps 1 --warmup 0 > $OUT/n64.json 2> $OUT/n64.err || exit 1
HGE_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --k 256 --steps 1 --warmup 0 > $OUT/n256.json 2> $OUT/n256.err || exit 1
grep stamps $OUT/*.err | tail -4
