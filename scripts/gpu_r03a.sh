#!/bin/bash
# round 3, first GPU pass: the new per-member rounds selection against the goldens,
# config 5 at size, then the default bench line and the Monte Carlo line
set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_golden.py tests/test_gpu_wide.py tests/test_gpu_split.py tests/test_gpu_mc.py > $O/pytest_a.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-secondary --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 400 python -u bench.py --workload mc --steps 3 --warmup 1 > $O/mc.json 2> $O/mc.err || exit 3
