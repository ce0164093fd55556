set -o pipefail
mkdir -p gpurun_out/mct
for T in 4 8 16; do
  timeout -k 10 300 python -u bench.py --workload mc --threads $T --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/mct/mc_t$T.json 2> gpurun_out/mct/mc_t$T.err || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/mct/mc_t$T.json').read().strip().splitlines()[-1]); print('threads $T', round(d['value']/1e6,2), d['ms_per_step'])"
done
