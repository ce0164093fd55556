"""Generate the committed golden vectors (tests/golden/*.npz, *.json).

Inputs are seeded synthetic submission streams (babble_amd.gossip) and the
reference's hand DAGs (tests/refdags.py); expected outputs come from the CPU
oracle (oracle/hg_oracle.cpp), which is itself pinned by the reference's
known-answer tests (tests/test_oracle_reference.py).  Re-run with
    python tests/golden/make_golden.py
Each npz holds the stream (creator, index, sp, op, ts, S, hash, ntx) -- or,
for the large ones, only the generator parameters `gen` (n, events, seed,
forkers, fork_p*1e6, cascade_p*1e6; tests regenerate the stream with
babble_amd.gossip.random_gossip) -- the call points, and the oracle's status,
order, per-call counts, rounds of every accepted event, witness flags, fame per
round slot, roundReceived / consensus timestamps, LCR/LCRE/transactions, the
oracle's DecideFame statistics (coin-branch evaluations, coin votes,
re-decided and flipped witnesses), and the witness-order invariance flags:
`order_invariant` / `fame_invariant` say whether R seeded random witness
iteration orders (Go's randomised map order, roundInfo.go:88-96; SURVEY.md
TL;DR 6) gave the same consensus order / the same fame of every witness as the
canonical ascending-creator order (`order_seeds` lists the seeds; empty = not
checked).
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
    # name, n, events, k, seed, forkers, fork_p, cascade_p, store_stream, order_seeds
    ("gossip_n4_e1000_k1", 4, 1000, 1, 1, 0, 0.0, 0.0, True, (1, 2, 3)),
    ("gossip_n4_e1000_k4", 4, 1000, 4, 1, 0, 0.0, 0.0, True, (1, 2, 3)),
    ("gossip_n4_e1000_oneshot", 4, 1000, 1000, 1, 0, 0.0, 0.0, True, (1, 2, 3)),
    ("gossip_n16_e3000_k16", 16, 3000, 16, 2, 0, 0.0, 0.0, True, (1, 2, 3)),
    ("gossip_n32_e2000_k32_forks", 32, 2000, 32, 3, 10, 0.05, 0.0, True, (1, 2, 3)),
    # config 5's forkers with cascades: events built on fork twins are rejected too
    ("gossip_n32_e3000_k32_cascade", 32, 3000, 32, 4, 10, 0.05, 0.5, True, (1, 2, 3)),
    # wide hashgraphs (N > 32: sweep coordinates + cooperative rounds); the
    # oracle takes 5-100 s on these, so the GPU tests compare against the file
    ("wide_n64_e8000_k64", 64, 8000, 64, 6, 0, 0.0, 0.0, True, ()),
    ("wide_n128_e15000_k128", 128, 15000, 128, 5, 0, 0.0, 0.0, True, ()),
    ("wide_n256_e25000_k256", 256, 25000, 256, 5, 0, 0.0, 0.0, True, ()),
    ("wide_n64_e100000_k64", 64, 100_000, 64, 8, 0, 0.0, 0.0, False, ()),
    ("wide_n256_e51200_k256", 256, 51_200, 256, 9, 0, 0.0, 0.0, False, ()),
]


def describe(o, dag, status, order, counts, calls):
    rounds, wit = o.event_rounds()
    rr, cts = o.event_received()
    st = o.stats()
    return dict(status=status, order=order, counts=counts, calls=calls, rounds=rounds, witness=wit.astype(np.int8),
                fame=o.fame_table(), rr=rr, cts=cts, undetermined=o.undetermined(),
                fame_stats=np.array([st["coin_evals"], st["coin_votes"], st["redecided"], st["flipped"]],
                                    np.int64),
                scalars=np.array([o.rounds(), -1 if o.last_consensus_round() is None else o.last_consensus_round(),
                                  o.last_committed_round_events(), o.consensus_transactions()],
                                 np.int64))


def order_invariance(dag, calls, order, fame, seeds):
    """Run the oracle under seeded random witness orders: (order same, fame same)."""
    same_order, same_fame = True, True
    acc = None
    for sd in seeds:
        o, status, order2, _ = replay(dag, calls, order_seed=sd)
        same_order &= bool(np.array_equal(order, order2))
        if acc is None:
            acc = status >= 0
        creators = dag["creator"][acc]
        R = o.rounds()
        f2 = np.full(fame.shape, -1, np.int8)
        for r in range(min(R, fame.shape[0])):
            for w in o.round_witnesses(r):
                f2[r, creators[w]] = o.round_fame(r, w)
        same_fame &= bool(np.array_equal(f2, fame)) and R == fame.shape[0]
    return same_order, same_fame


def main(only=None):
    for name, n, events, k, seed, fk, fp, cp, keep, seeds in CASES:
        if only and only not in name:
            continue
        dag = random_gossip(n, events, seed=seed, forkers=fk, fork_p=fp, cascade_p=cp)
        calls = schedule(len(dag["creator"]), k)
        o, status, order, counts = replay(dag, calls)
        out = describe(o, dag, status, order, counts, calls)
        inv_o, inv_f = order_invariance(dag, calls, order, out["fame"], seeds) if seeds else (False, False)
        out["order_seeds"] = np.array(seeds, np.int64)
        out["order_invariant"] = np.bool_(inv_o)
        out["fame_invariant"] = np.bool_(inv_f)
        stream = {k2: dag[k2] for k2 in ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")}
        gen = np.array([n, events, seed, fk, round(fp * 1e6), round(cp * 1e6)], np.int64)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), n=np.int32(n), gen=gen,
                            **(stream if keep else {}), **out)
        print(name, "ordered", len(order), "rounds", out["scalars"][0], "fame stats",
              out["fame_stats"].tolist(), "invariant (order, fame)", (inv_o, inv_f) if seeds else "-")
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
