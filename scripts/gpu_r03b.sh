#!/bin/bash
# rounds-kernel iteration: wide parity tests, the default bench line, section stamps at 256/2M
set -o pipefail
O=gpurun_out/${1:-r03b}
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_golden.py tests/test_gpu_wide.py tests/test_gpu_split.py tests/test_gpu_store.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 2
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['parity']); print(list(d['kernels_ms_per_replay'].items())[:6])"
bash scripts/gpu_stamps.sh ${1:-r03b}_st
