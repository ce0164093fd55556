"""Oracle digests of every graph of config 5's Monte Carlo batch (test infrastructure).

bench.py --workload mc replays graph g (0 <= g < 1024) from the seeded stream
random_gossip(32, 10000, seed=1 + g, forkers=10, fork_p=0.05, cascade_p=0.5)
with RunConsensus every K = 32 submissions.  This script runs the CPU oracle
(oracle/hg_oracle.cpp, the Go-faithful restatement pinned by the reference's
known-answer tests) on each graph and stores the full-state digest of
tests/golden/digest.py, so the bench and the GPU tests check EVERY graph of the
batch bit-exactly (order, batches, rounds, witnesses, fame, round received,
consensus timestamps, undetermined list, scalars) without running the oracle.

    python tests/golden/make_mc_digests.py [graphs] [procs]
"""
import json
import os
import sys
import time
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

PARAMS = dict(n=32, events=10_000, k=32, seed0=1, forkers=10, fork_p=0.05, cascade_p=0.5)
OUT = os.path.join(HERE, "mc_n32_e10000_k32_digests.json")


def graph_stream(g, p=PARAMS):
    from babble_amd.gossip import random_gossip, schedule
    dag = random_gossip(p["n"], p["events"], seed=p["seed0"] + g, forkers=p["forkers"], fork_p=p["fork_p"],
                        cascade_p=p["cascade_p"])
    return dag, schedule(len(dag["creator"]), p["k"])


def oracle_state(dag, calls):
    from make_golden import describe
    from oracle.oracle import replay
    o, status, order, counts = replay(dag, calls)
    d = describe(o, dag, status, order, counts, calls)
    return {k: d[k] for k in ("status", "order", "counts", "rounds", "witness", "fame", "rr", "cts",
                              "undetermined", "scalars")}


def one(g):
    from digest import digest
    dag, calls = graph_stream(g)
    st = oracle_state(dag, calls)
    return digest(st), int(len(st["order"])), int((st["status"] < 0).sum())


def main():
    graphs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    t = time.time()
    with Pool(procs) as pool:
        res = pool.map(one, range(graphs), chunksize=4)
    out = {"params": PARAMS, "graphs": graphs, "digests": [r[0] for r in res],
           "ordered": [r[1] for r in res], "rejected": [r[2] for r in res]}
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"{OUT}: {graphs} graphs, {sum(out['ordered'])} ordered, {sum(out['rejected'])} rejected "
          f"({time.time() - t:.1f} s)")


if __name__ == "__main__":
    main()
