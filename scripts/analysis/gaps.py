"""Idle time between consecutive device operations of one replay (rocprofv3
--kernel-trace --memory-copy-trace CSVs): where a 256/10M step spends the time
its kernels do not account for.  Usage: gaps.py <rocprofv3 output dir>."""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d):
    ops = []
    for r in rows(d, "*kernel_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], "k"))
    for r in rows(d, "*memory_copy_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?"), "c"))
    ops.sort()
    if not ops:
        print("no operations")
        return
    # the last replay: from the last k_reset_rounds (a fresh replay's first kernel) on
    starts = [i for i, o in enumerate(ops) if "k_reset_rounds" in o[2]]
    i0 = starts[-1] if starts else 0
    seg = ops[i0:]
    t0, t1 = seg[0][0], max(o[1] for o in seg)
    busy = 0
    gaps = defaultdict(lambda: [0, 0])
    end = seg[0][0]
    for s, e, name, _ in seg:
        if s > end:
            g = gaps[name]
            g[0] += s - end
            g[1] += 1
        busy += max(0, e - max(s, end))
        end = max(end, e)
    print(f"last replay: {(t1 - t0) / 1e6:.3f} ms span, {busy / 1e6:.3f} ms busy, {len(seg)} ops")
    print("idle before each op (ms, count):")
    for name, (ns, n) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:30]:
        print(f"  {ns / 1e6:8.3f} {n:6d}  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
