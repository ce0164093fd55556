#!/bin/bash
# online per-call path timings (host round trips, p50/p99) on one GPU
set -o pipefail
mkdir -p gpurun_out/online
timeout -k 10 600 python -u scripts/online_probe.py "$@" > gpurun_out/online/online.json 2> gpurun_out/online/online.err
rc=$?
cat gpurun_out/online/online.json
tail -5 gpurun_out/online/online.err
exit $rc
