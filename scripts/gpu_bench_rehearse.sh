#!/bin/bash
# bench.py --gpus 2 rehearsed on the one GPU of the box (two ranks share it, gloo): the
# sharded split's bench path end to end (parity on rank 0, replicas line); timings
# are not meaningful (the ranks compete for one GPU)
set -o pipefail
OUT=gpurun_out/${1:-rehearse}
mkdir -p $OUT
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || { tail -30 $OUT/bench2.err; exit 1; }
python -c "
import json
d=json.loads(open('$OUT/bench2.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['scaling'], round(d['value']/1e6,2), d['ms_per_step'], d['config']['parallelism'][:40], d.get('split_fallbacks'), d['parity'][:60])
print(d.get('secondary'))"
