"""Generate the committed golden vectors (tests/golden/*.npz, *.json).

Inputs are seeded synthetic submission streams (babble_amd.gossip) and the
reference's hand DAGs (tests/refdags.py); expected outputs come from the CPU
oracle (oracle/hg_oracle.cpp), which is itself pinned by the reference's
known-answer tests (tests/test_oracle_reference.py).  Re-run with
    python tests/golden/make_golden.py
Each npz holds the stream (creator, index, sp, op, ts, S, hash, ntx), the
call points, and the oracle's status, order, per-call counts, rounds of every
accepted event, witness flags, fame per round slot, LCR/LCRE/transactions.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from babble_amd.gossip import random_gossip, schedule  # noqa: E402
from oracle.oracle import replay  # noqa: E402
from refdags import CONSENSUS_DAG, ROUND_DAG, SMALL_DAG, to_stream  # noqa: E402

CASES = [
    # name, n, events, k, seed, forkers, fork_p
    ("gossip_n4_e1000_k1", 4, 1000, 1, 1, 0, 0.0),
    ("gossip_n4_e1000_k4", 4, 1000, 4, 1, 0, 0.0),
    ("gossip_n4_e1000_oneshot", 4, 1000, 1000, 1, 0, 0.0),
    ("gossip_n16_e3000_k16", 16, 3000, 16, 2, 0, 0.0),
    ("gossip_n32_e2000_k32_forks", 32, 2000, 32, 3, 10, 0.05),
    # wide hashgraphs (N > 32: sweep coordinates + cooperative rounds); the
    # oracle takes 5-40 s on these, so the GPU tests compare against the file
    ("wide_n64_e8000_k64", 64, 8000, 64, 6, 0, 0.0),
    ("wide_n128_e15000_k128", 128, 15000, 128, 5, 0, 0.0),
    ("wide_n256_e25000_k256", 256, 25000, 256, 5, 0, 0.0),
]


def describe(o, dag, status, order, counts, calls):
    acc = status >= 0
    ids = status[acc]
    E = len(ids)
    rounds = np.array([o.round(int(x)) for x in range(E)], np.int32)
    wit = np.array([o.witness(int(x)) for x in range(E)], np.int8)
    creators = dag["creator"][acc]
    R = o.rounds()
    fame = np.full((R, dag["n"]), -1, np.int8)
    for r in range(R):
        for w in o.round_witnesses(r):
            fame[r, creators[w]] = o.round_fame(r, w)
    rr = np.array([o.round_received(int(x)) if o.round_received(int(x)) is not None else -1
                   for x in range(E)], np.int32)
    cts = np.array([o.consensus_timestamp(int(x)) if rr[x] >= 0 else 0 for x in range(E)], np.int64)
    return dict(status=status, order=order, counts=counts, calls=calls, rounds=rounds, witness=wit,
                fame=fame, rr=rr, cts=cts, undetermined=o.undetermined(),
                scalars=np.array([R, -1 if o.last_consensus_round() is None else o.last_consensus_round(),
                                  o.last_committed_round_events(), o.consensus_transactions()],
                                 np.int64))


def main(only=None):
    for name, n, events, k, seed, fk, fp in CASES:
        if only and only not in name:
            continue
        dag = random_gossip(n, events, seed=seed, forkers=fk, fork_p=fp)
        calls = schedule(len(dag["creator"]), k)
        o, status, order, counts = replay(dag, calls)
        out = describe(o, dag, status, order, counts, calls)
        stream = {k2: dag[k2] for k2 in ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), n=np.int32(n), **stream, **out)
        print(name, "ordered", len(order), "rounds", out["scalars"][0])
    if only:
        return
    # reference hand DAGs: names, expected results (by name)
    ref = {}
    for nm, dag in (("small", SMALL_DAG), ("round", ROUND_DAG), ("consensus", CONSENSUS_DAG)):
        s, ix = to_stream(dag)
        o, status, order, counts = replay(s, [len(dag)])
        names = {v: k2 for k2, v in ix.items()}
        ref[nm] = {
            "events": [[d[0], d[1], d[2], d[3]] for d in dag],
            "order_one_shot": [names[int(i)] for i in order],
            "rounds": {names[x]: o.round(x) for x in range(len(dag))},
            "witness": {names[x]: bool(o.witness(x)) for x in range(len(dag))},
            "last_consensus_round": o.last_consensus_round(),
        }
    with open(os.path.join(HERE, "reference_dags.json"), "w") as f:
        json.dump(ref, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
