#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) -> profiles/pmc_traffic.json
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
python3 scripts/pmc_traffic.py $OUT/n16 gossip_n16_e100000_k16 -- --steps 1 --warmup 0 > $OUT/n16.log 2>&1 || { tail -30 $OUT/n16.log; exit 1; }
python3 scripts/pmc_traffic.py $OUT/n256 gossip_n256_e2000000_k256 -- --steps 1 --warmup 0 --participants 256 --events 2000000 > $OUT/n256.log 2>&1 || { tail -30 $OUT/n256.log; exit 1; }
cp profiles/pmc_traffic.json $OUT/
tail -40 $OUT/n16.log
