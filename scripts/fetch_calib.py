"""Calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte counts on gfx950
(run on the GPU box; build/fetch_calib is built beforehand from
scripts/ubench/fetch_calib.hip, the recipe in its header).

usage: python scripts/fetch_calib.py <out_dir> [--parse-only]
Two counter passes (FETCH_SIZE, then WRITE_SIZE), each its own rocprofv3 run with
--kernel-trace only.  Writes <out_dir>/fetch_calib.json:
  {"read": {width: bytes / (FETCH_SIZE KiB * 1024)}, "write": {width: bytes / (WRITE_SIZE * 1024)}}
i.e. the factor to multiply a counter by to get bytes, per access width (bytes per lane).
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BYTES = 1 << 30
# kernel name (as rocprofv3 prints it) -> (direction, bytes per lane)
KERNELS = {"k_read<unsigned short>": ("read", 2), "k_read<unsigned int>": ("read", 4),
           "k_read<HIP_vector_type<unsigned int, 2u> >": ("read", 8),
           "k_read<HIP_vector_type<unsigned int, 4u> >": ("read", 16),
           "k_write<unsigned int>": ("write", 4), "k_write<HIP_vector_type<unsigned int, 2u> >": ("write", 8),
           "k_write<HIP_vector_type<unsigned int, 4u> >": ("write", 16)}


def classify(name):
    name = name.replace("void ", "").split("(")[0].strip()
    for k, v in KERNELS.items():
        if name == k:
            return v
    if name.startswith("k_read") or name.startswith("k_write"):
        # an unexpected spelling of the vector types: fall back on the template argument
        d = "read" if name.startswith("k_read") else "write"
        w = 2 if "short" in name else 16 if "4u" in name else 8 if "2u" in name else 4
        return d, w
    return None


def run_pass(out_dir, counter, parse_only):
    d = os.path.join(out_dir, counter.lower())
    if not parse_only:
        subprocess.check_call(["timeout", "-s", "KILL", "60", "rocprofv3", "--kernel-trace", "--pmc", counter,
                               "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                               os.path.join(ROOT, "build", "fetch_calib")], cwd=ROOT)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    res = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            c = classify(row["Kernel_Name"])
            if c:
                res[c] = res.get(c, 0.0) + float(row["Counter_Value"])
    return res


def main():
    out_dir = sys.argv[1]
    parse_only = "--parse-only" in sys.argv
    fetch = run_pass(out_dir, "FETCH_SIZE", parse_only)
    write = run_pass(out_dir, "WRITE_SIZE", parse_only)
    out = {"bytes_per_kernel": BYTES, "read": {}, "write": {}, "raw_kib": {}}
    for (d, w), v in sorted(fetch.items()):
        if d == "read":
            out["read"][str(w)] = round(BYTES / (v * 1024), 4) if v else None
            out["raw_kib"][f"read{w}_FETCH_SIZE"] = v
    for (d, w), v in sorted(write.items()):
        if d == "write":
            out["write"][str(w)] = round(BYTES / (v * 1024), 4) if v else None
            out["raw_kib"][f"write{w}_WRITE_SIZE"] = v
    out["note"] = ("factor = known bytes / counter bytes per access width (bytes per lane); "
                   "multiply a kernel's counter by the factor of its load / store width")
    json.dump(out, open(os.path.join(out_dir, "fetch_calib.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
