#!/bin/bash
# SQ counters of the batch engine's kernels (bench.py --workload mc), one rocprofv3 pass.
# usage: scripts/gpu_pmc_mc.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_mc}
shift
ARGS=${*:---graphs 1024}
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $OUT/sq -o pmc -- \
  python3 bench.py --workload mc --no-cpu-baseline --steps 1 --warmup 0 --ramp-s 0 $ARGS > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
per = {}
for f in glob.glob(os.path.join(sys.argv[1], "sq", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        k = per.setdefault(name, {})
        k[row["Counter_Name"]] = k.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
for nm, s in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    wc = max(s.get("SQ_WAVE_CYCLES", 0), 1)
    print(f"{nm[:50]:50s} wave_cycles={wc:.3g} wait={s.get('SQ_WAIT_ANY',0)/wc:.2f} "
          f"issue_stall={s.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active={s.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
          f"lds_stall={s.get('SQ_WAIT_INST_LDS',0)/wc:.2f} valu={s.get('SQ_INSTS_VALU',0):.3g} "
          f"lds={s.get('SQ_INSTS_LDS',0):.3g} salu={s.get('SQ_INSTS_SALU',0):.3g}")
PY
