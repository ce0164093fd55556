#!/bin/bash
# Exploratory sweep: chunk length and larger configurations.
set -o pipefail
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
for L in 256 512 1024; do
  HGE_CHUNK=$L timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/chunk_$L.json 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 64 --events 1000000 --k 64 --steps 3 --warmup 1 > $OUT/n64_1m.json 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants 256 --events 1000000 --k 256 --steps 2 --warmup 1 > $OUT/n256_1m.json 2>&1 || exit 1
