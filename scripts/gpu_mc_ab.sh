#!/bin/bash
# config 5 (Monte Carlo, N = 32): build/libhge_n32.so (block-per-pair fame for every N >= 32) vs
# build/libhge.so, then that variant through the MC, golden and parity GPU tests
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mcab}
mkdir -p $OUT
for L in build/libhge_n32.so build/libhge.so build/libhge_n32.so build/libhge.so; do
  T=$(basename $L .so)
  HGE_LIB=$L timeout -k 10 300 python -u bench.py --workload mc --no-cpu-baseline --steps 3 --warmup 1 > $OUT/mc_$T.json 2> $OUT/mc_$T.err || { tail -20 $OUT/mc_$T.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/mc_$T.json').read().strip().splitlines()[-1])
print('$T mc', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:60], [kv for kv in d['kernels_ms_per_replay'].items() if 'fame_decide' in kv[0]])"
done
HGE_LIB=build/libhge_n32.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_mc.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_wide.py > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAIL|Error" $OUT/pytest.log | head -20; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
