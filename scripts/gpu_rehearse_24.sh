#!/bin/bash
# bench.py --gpus 2 and --gpus 4 rehearsed on the one GPU of the box (ranks share it, gloo): the sharded
# split's bench path end to end (parity on rank 0, replicas line); timings are not meaningful
set -o pipefail
OUT=gpurun_out/${1:-rehearse24}
mkdir -p $OUT
for W in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2951$W bench.py --gpus $W --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench$W.json 2> $OUT/bench$W.err || { tail -30 $OUT/bench$W.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/bench$W.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['scaling'], round(d['value']/1e6,2), d['ms_per_step'], d['config']['parallelism'][:40], d.get('split_fallbacks'), d['parity'][:60])
print(d.get('secondary'))"
done
