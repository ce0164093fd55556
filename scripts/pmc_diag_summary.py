"""Summarise scripts/gpu_pmc_diag.sh output: per kernel, each counter summed over
its launches (and the launch count), for the kernels that take the most wave cycles."""
import csv
import glob
import os
import sys


def load(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("hge::", "").strip()
            k = per.setdefault(name, {})
            c = row["Counter_Name"]
            v, n = k.get(c, (0.0, 0))
            k[c] = (v + float(row["Counter_Value"]), n + 1)
    return per


def main():
    out = sys.argv[1]
    tcc, sq = load(os.path.join(out, "tcc")), load(os.path.join(out, "sq"))
    names = sorted(sq, key=lambda k: -sq[k].get("SQ_WAVE_CYCLES", (0, 0))[0])[:12]
    for nm in names:
        s, t = sq.get(nm, {}), tcc.get(nm, {})
        g = lambda d, c: d.get(c, (0.0, 0))[0]
        hit, miss = g(t, "TCC_HIT_sum"), g(t, "TCC_MISS_sum")
        wc = max(g(s, "SQ_WAVE_CYCLES"), 1.0)
        print(f"{nm[:60]:60s} launches={s.get('SQ_WAVE_CYCLES', (0, 0))[1]} "
              f"L2hit={hit / max(hit + miss, 1):.3f} rdreq={g(t, 'TCC_EA0_RDREQ_sum'):.3g} "
              f"wait={g(s, 'SQ_WAIT_ANY') / wc:.2f} issue_stall={g(s, 'SQ_WAIT_INST_ANY') / wc:.2f} "
              f"active={g(s, 'SQ_ACTIVE_INST_ANY') / wc:.2f} lds_stall={g(s, 'SQ_WAIT_INST_LDS') / wc:.2f} "
              f"valu={g(s, 'SQ_INSTS_VALU'):.3g} lds={g(s, 'SQ_INSTS_LDS'):.3g} salu={g(s, 'SQ_INSTS_SALU'):.3g} "
              f"wave_cycles={wc:.3g}")


if __name__ == "__main__":
    main()
