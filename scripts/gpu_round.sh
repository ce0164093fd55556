#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel-trace summary.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-run}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*stats*' | head
