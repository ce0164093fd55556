#!/bin/bash
# iteration pass: wide-path parity (goldens, wide, store, split), then the default bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 700 $PYT tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_store.py tests/test_gpu_split.py tests/test_gpu_reference.py tests/test_gpu_replay_paths.py > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAIL|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
python -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), 'Mev/s', d['ms_per_step'], 'ms', d['parity'])
print(list(d['kernels_ms_per_replay'].items())[:9])"
