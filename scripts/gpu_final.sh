#!/bin/bash
# the round-end invocations as the driver runs them: smoke, then the default bench line
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 2; }
python -c "
import json
d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:200]); print(d['cpu_baseline']['value'], d['roofline']['frac'])
for k,v in d['secondary'].items(): print(k, v.get('value'), v.get('call_latency_us'), v.get('host_round_trips_per_call'), (v.get('parity') or '')[:40])"
