"""Regenerate committed goldens with the oracle and compare them field by field
(test infrastructure).

    python tests/golden/regen_check.py [--scale] [--release LAG] [name-substring ...]

Used to re-pin the oracle after a change: every golden must come out
byte-identical in the faithful mode and in the scale mode (hg_oracle.cpp
header).  The bench prefixes are regenerated from their generator parameters
(`prefix`, `n`, `events`, `k`, `seed`).
"""
import argparse
import glob
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from babble_amd.gossip import random_gossip, schedule  # noqa: E402
from make_golden import describe  # noqa: E402
from oracle.oracle import replay  # noqa: E402

FIELDS = ("status", "order", "counts", "rounds", "witness", "fame", "rr", "cts", "undetermined", "scalars",
          "fame_stats")


def stream_of(g):
    if "creator" in g.files:
        dag = {k: g[k] for k in ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")}
        dag["n"] = int(g["n"])
        return dag, g["calls"]
    if "prefix" in g.files:
        n, E, K, seed, P = (int(g[k]) for k in ("n", "events", "k", "seed", "prefix"))
        dag = random_gossip(n, E, seed=seed)
        sub = {k: (v[:P] if isinstance(v, np.ndarray) else v) for k, v in dag.items()}
        return sub, schedule(P, K)
    n, E, seed, fk, fp, cp = (int(v) for v in g["gen"])
    dag = random_gossip(n, E, seed=seed, forkers=fk, fork_p=fp / 1e6, cascade_p=cp / 1e6)
    return dag, g["calls"]


def check(path, scale, release):
    g = np.load(path, allow_pickle=False)
    dag, calls = stream_of(g)
    t = time.time()
    o, status, order, counts = replay(dag, calls, scale=scale, release_lag=release)
    d = describe(o, dag, status, order, counts, calls)
    d["order"] = d["order"].astype(np.int32)
    dt = time.time() - t
    bad = []
    for k in FIELDS:
        if k not in g.files:
            continue
        a, b = np.asarray(d[k]), g[k]
        if k == "status" and "prefix" in g.files:
            continue
        if a.shape != b.shape or not np.array_equal(a.astype(b.dtype), b):
            bad.append(k)
    if "status" not in g.files or "prefix" in g.files:
        assert (status >= 0).all()
    return bad, dt, len(order)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", action="store_true")
    ap.add_argument("--release", type=int, default=-1)
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    paths = sorted(glob.glob(os.path.join(HERE, "*.npz")))
    if a.names:
        paths = [p for p in paths if any(s in os.path.basename(p) for s in a.names)]
    ok = True
    for p in paths:
        bad, dt, m = check(p, a.scale, a.release)
        ok &= not bad
        print(f"{os.path.basename(p)}: {'OK' if not bad else 'DIFF ' + ','.join(bad)} "
              f"({m} ordered, {dt:.1f} s)", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
