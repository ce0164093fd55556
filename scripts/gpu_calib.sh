#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (known-byte kernels), then the default bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-calib}
mkdir -p $OUT
timeout -k 10 200 python -u scripts/fetch_calib.py $OUT > $OUT/calib.log 2>&1 || { tail -30 $OUT/calib.log; exit 1; }
tail -1 $OUT/calib.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
python -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['ms_per_step'], d['parity'], d.get('admission_ms'))
for k,v in d['secondary'].items(): print(k, v.get('value'), v.get('call_latency_us'), v.get('host_round_trips_per_call'), v.get('parity'))"
