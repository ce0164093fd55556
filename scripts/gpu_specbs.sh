#!/bin/bash
# walker block size 512 (2 per CU) vs 1024 (1 per CU): parity at 1024, then 64/1M and 128/1M over seeds
set -o pipefail
OUT=gpurun_out/${1:-specbs}
mkdir -p $OUT
HGE_COOP_SPEC_BS=1024 timeout -k 10 400 python -u -m pytest tests/test_gpu_coop_spec.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest1024.log 2>&1 || { tail -30 $OUT/pytest1024.log; exit 1; }
tail -1 $OUT/pytest1024.log
run() {  # n bs seed
HGE_COOP_SPEC_BS=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --participants $1 --events 1000000 --steps 2 --warmup 1 --seed $3 > $OUT/n$1_bs$2_s$3.json 2> $OUT/n$1_bs$2_s$3.err || { tail -5 $OUT/n$1_bs$2_s$3.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/n$1_bs$2_s$3.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('n$1 bs$2 s$3', round(d['value']/1e6,2), d['ms_per_step'], k.get('k_rounds_coop_spec'))
"
}
for s in 1 2 3; do run 64 512 $s && run 64 1024 $s && run 128 512 $s && run 128 1024 $s || exit 1; done
