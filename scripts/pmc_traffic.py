"""HBM traffic per kernel launch from rocprofv3 PMC passes (run on the GPU box).

usage: python scripts/pmc_traffic.py <out_dir> <config-key> [--parse-only] -- <bench args...>
Runs two counter passes over `python3 bench.py <bench args>` (FETCH_SIZE, then
WRITE_SIZE: they cannot share one pass on gfx950), each in its own rocprofv3
run with --kernel-trace only, parses counter_collection.csv and merges
{config-key: {kernel: {fetch_bytes, write_bytes, bytes_per_launch, launches}}}
into profiles/<round>/pmc_traffic.json (ROUND below).  FETCH_SIZE is reported in KiB and, on gfx950,
counts half of the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM),
so it is doubled; WRITE_SIZE (KiB) is taken as is.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


ROUND = "r06"  # the profiles/ directory this round's passes go to

def run_pass(out_dir, counter, bench_args, parse_only=False):
    d = os.path.join(out_dir, counter.lower())
    if not parse_only:
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--kernel-trace", "--pmc", counter,
               "--output-format", "csv", "-d", d, "-o", "pmc", "--", "python3", "bench.py",
               "--no-cpu-baseline", "--no-secondary", "--profile-steps", "1"] + bench_args
        subprocess.check_call(cmd, cwd=ROOT)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("hge::", "").replace("hgb::", "")
            name = name.split("<")[0].strip()
            v = float(row["Counter_Value"])
            s = per.setdefault(name, [0.0, 0])
            s[0] += v
            s[1] += 1
    return per


def main():
    out_dir, key = sys.argv[1], sys.argv[2]
    bench_args = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
    parse_only = "--parse-only" in sys.argv[:sys.argv.index("--") if "--" in sys.argv else None]
    fetch = run_pass(out_dir, "FETCH_SIZE", bench_args, parse_only)
    write = run_pass(out_dir, "WRITE_SIZE", bench_args, parse_only)
    res = {}
    # every replay fills the chain table once (k_chain_fill): the replay count
    # (k_reset_rounds also runs at prepare time)
    # (the batch engine: kb_coords, once per batch replay)
    replays = max(1, fetch.get("k_chain_fill", fetch.get("kb_coords", [0.0, 0]))[1])
    for name in sorted(set(fetch) | set(write)):
        fb, fl = fetch.get(name, [0.0, 0])
        wb, wl = write.get(name, [0.0, 0])
        launches = max(fl, wl, 1)
        fetch_b = 2.0 * fb * 1024 / max(fl, 1)
        write_b = wb * 1024 / max(wl, 1)
        # per replay: every launch of the replay, the queued sweeps that returned at once included
        per_replay = (2.0 * fb + wb) * 1024 / replays
        res[name] = {"fetch_bytes": round(fetch_b), "write_bytes": round(write_b),
                     "bytes_per_launch": round(fetch_b + write_b), "launches": launches,
                     "bytes_per_replay": round(per_replay), "replays": replays}
    path = os.path.join(ROOT, "profiles", ROUND, "pmc_traffic.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    try:
        allres = json.load(open(path))
    except (OSError, ValueError):
        allres = {}
    if "configs" in allres and "round" not in allres:
        allres = {}  # an older round's file: start this round's afresh
    allres["round"] = ROUND
    allres.setdefault("note", "HBM bytes per launch from rocprofv3 FETCH_SIZE (x2, gfx950) + "
                              "WRITE_SIZE, separate passes (scripts/pmc_traffic.py)")
    allres.setdefault("configs", {})[key] = res
    json.dump(allres, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: res}, indent=1))


if __name__ == "__main__":
    main()
