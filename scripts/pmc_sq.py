"""Per-kernel SQ counters from one rocprofv3 PMC pass (run on the GPU box).

usage: python scripts/pmc_sq.py <out_dir> [--parse-only] [--counters A,B,..] -- <bench args...>
One pass of 8 SQ counters over `python3 bench.py <bench args>` with --kernel-trace
only; prints, per kernel and launch, waves, wave-cycles, the share of wave-cycles
spent waiting on an instruction dependency (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES) and
the instruction mix.
"""
import csv
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU",
            "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE"]


def main():
    out_dir = sys.argv[1]
    bench_args = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
    parse_only = "--parse-only" in sys.argv
    counters = COUNTERS
    if "--counters" in sys.argv:
        counters = sys.argv[sys.argv.index("--counters") + 1].split(",")
    d = os.path.join(out_dir, "sq")
    if not parse_only:
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--kernel-trace", "--pmc"] + counters + [
            "--output-format", "csv", "-d", d, "-o", "pmc", "--", "python3", "bench.py",
            "--no-cpu-baseline", "--profile-steps", "1", "--ramp-s", "0"] + bench_args
        subprocess.check_call(cmd, cwd=ROOT)
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("hge::", "").strip()
            k = per.setdefault(name, {})
            c = row["Counter_Name"]
            k.setdefault(c, []).append(float(row["Counter_Value"]))
    rows = []
    for name, k in per.items():
        n = max(len(v) for v in k.values())
        avg = {c: sum(v) / max(len(v), 1) for c, v in k.items()}
        rows.append((avg.get("SQ_WAVE_CYCLES", 0), name, n, avg))
    rows.sort(reverse=True)
    print(f"{'kernel':40s} {'launch':>6s} {'waves':>8s} {'wavecyc':>10s} {'wait%':>6s} "
          f"{'valu/w':>7s} {'vmem/w':>7s} {'salu/w':>7s} {'lds/w':>6s} {'gpu_cyc':>9s}")
    extra = [c for c in counters if c not in COUNTERS]
    for wc, name, n, a in rows[:30]:
        if extra:
            print(f"{name[:40]:40s} " + " ".join(f"{c}={a.get(c, 0):.0f}" for c in ["SQ_WAVES", "SQ_WAVE_CYCLES"] + extra))
            continue
        w = max(a.get("SQ_WAVES", 1), 1)
        print(f"{name[:40]:40s} {n:6d} {w:8.0f} {wc:10.0f} "
              f"{100 * a.get('SQ_WAIT_INST_ANY', 0) / max(wc, 1):6.1f} "
              f"{a.get('SQ_INSTS_VALU', 0) / w:7.1f} {a.get('SQ_INSTS_VMEM_RD', 0) / w:7.1f} "
              f"{a.get('SQ_INSTS_SALU', 0) / w:7.1f} {a.get('SQ_INSTS_LDS', 0) / w:6.1f} "
              f"{a.get('GRBM_GUI_ACTIVE', 0):9.0f}")


if __name__ == "__main__":
    main()
