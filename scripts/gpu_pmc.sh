#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) -> profiles/r06/pmc_traffic.json
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
timeout -k 10 500 python3 scripts/pmc_traffic.py $OUT/n256 gossip_n256_e10000000_k256 -- --steps 1 --warmup 0 --ramp-s 0 > $OUT/n256.log 2>&1 || { tail -30 $OUT/n256.log; exit 1; }
timeout -k 10 300 python3 scripts/pmc_traffic.py $OUT/n16 gossip_n16_e100000_k16 -- --steps 1 --warmup 0 --participants 16 --events 100000 > $OUT/n16.log 2>&1 || { tail -30 $OUT/n16.log; exit 1; }
timeout -k 10 300 python3 scripts/pmc_traffic.py $OUT/mc mc_n32_e10000_k32_g1024 -- --workload mc --graphs 1024 --steps 1 --warmup 0 --ramp-s 0 > $OUT/mc.log 2>&1 || { tail -30 $OUT/mc.log; exit 1; }
cp profiles/r06/pmc_traffic.json $OUT/
python3 -c "
import json; d=json.load(open('profiles/r06/pmc_traffic.json'))['configs']['gossip_n256_e10000000_k256']
for k,v in sorted(d.items(), key=lambda kv:-kv[1]['bytes_per_replay'])[:10]: print(k, v)"
