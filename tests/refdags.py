"""The reference's hand-built hashgraphs, restated as data.

Each DAG is a list of (name, creator, self_parent_name, other_parent_name) in the
reference's insertion order.  Event creation order = list order, so the
synthetic timestamps (creation index * 1000 ns) reproduce the reference's
time.Now() ordering.  Hashes/S are fixed synthetic bytes (the reference draws
them from crypto/rand, so tests there assert by name only).

Sources:
  ROUND_DAG      hashgraph/hashgraph_test.go:324-369   (initRoundHashgraph)
  SMALL_DAG      hashgraph/hashgraph_test.go:78-129    (initHashgraph)
  CONSENSUS_DAG  hashgraph/hashgraph_test.go:835-950   (initConsensusHashgraph)
  PLAYBOOK       node/core_test.go:339-387, node/node_test.go:336-391
"""
import hashlib

import numpy as np

SMALL_DAG = [
    ("e0", 0, None, None), ("e1", 1, None, None), ("e2", 2, None, None),
    ("e01", 0, "e0", "e1"),
    ("e20", 2, "e2", "e01"),
    ("e12", 1, "e1", "e20"),
]

ROUND_DAG = [
    ("e0", 0, None, None), ("e1", 1, None, None), ("e2", 2, None, None),
    ("e10", 1, "e1", "e0"),
    ("e21", 2, "e2", "e10"),
    ("e02", 0, "e0", "e21"),
    ("f1", 1, "e10", "e02"),
]

CONSENSUS_DAG = ROUND_DAG + [
    ("f0", 0, "e02", "f1"),
    ("f2", 2, "e21", "f1"),
    ("f10", 1, "f1", "f0"),
    ("f21", 2, "f2", "f10"),
    ("f02", 0, "f0", "f21"),
    ("g1", 1, "f10", "f02"),
    ("g0", 0, "f02", "g1"),
    ("g2", 2, "f21", "g1"),
    ("g10", 1, "g1", "g0"),
    ("g21", 2, "g2", "g10"),
    ("g02", 0, "g0", "g21"),
    ("h1", 1, "g10", "g02"),
    ("h0", 0, "g02", "h1"),
    ("h2", 2, "g21", "h1"),
]

# (from, to, payload) of node/core_test.go:343-362; in core_test the `to` core pulls and
# creates the new event, in node_test.go:340-359 the same DAG is built with the roles named
# the other way round (`from` pulls).  Here: puller, peer.
PLAYBOOK = [
    (1, 0, "e10"), (2, 1, "e21"), (0, 2, "e02"), (1, 0, "f1"), (0, 1, "f0"), (2, 1, "f2"),
    (1, 0, "f10"), (2, 1, "f21"), (0, 2, "f02"), (1, 0, "g1"), (0, 1, "g0"), (2, 1, "g2"),
    (1, 0, "g10"), (2, 1, "g21"), (0, 2, "g02"), (1, 0, "h1"), (0, 1, "h0"), (2, 1, "h2"),
]

TS_BASE = 1_500_000_000_000_000_000


def fixed_bytes(name, salt):
    return hashlib.sha256(f"{salt}:{name}".encode()).digest()


def to_stream(dag):
    """Submission-stream dict (same layout as babble_amd.gossip) + name->index map."""
    names = [d[0] for d in dag]
    pos = {nm: i for i, nm in enumerate(names)}
    n = 1 + max(d[1] for d in dag)
    E = len(dag)
    out = {
        "n": n,
        "creator": np.array([d[1] for d in dag], np.int32),
        "sp": np.array([pos[d[2]] if d[2] else -1 for d in dag], np.int32),
        "op": np.array([pos[d[3]] if d[3] else -1 for d in dag], np.int32),
        "ts": TS_BASE + 1000 * np.arange(E, dtype=np.int64),
        "S": np.frombuffer(b"".join(fixed_bytes(nm, "S") for nm in names), np.uint8).reshape(E, 32).copy(),
        "hash": np.frombuffer(b"".join(fixed_bytes(nm, "H") for nm in names), np.uint8).reshape(E, 32).copy(),
        "ntx": np.zeros(E, np.int32),
    }
    seq = {}
    idx = []
    for d in dag:
        idx.append(seq.get(d[1], 0))
        seq[d[1]] = idx[-1] + 1
    out["index"] = np.array(idx, np.int32)
    return out, pos


def playbook_views(n=3):
    """Simulate the three-core playbook and return, per core, its insertion order
    (list of global event names) and the RunConsensus points (after its own inserts).

    Core.Sync (node/core.go:134-157): the puller inserts the peer's unknown events in the
    peer's topological (insertion) order, then creates its own event (self head, peer head)
    and runs consensus.
    """
    events = {}            # name -> (creator, sp, op)
    order = []             # global creation order of names
    store = [[] for _ in range(n)]  # per-core insertion order
    head = {}
    for i in range(n):
        nm = f"e{i}"
        events[nm] = (i, None, None)
        order.append(nm)
        store[i].append(nm)
        head[i] = nm
    calls = [[] for _ in range(n)]
    txs = {}
    for puller, peer, name in PLAYBOOK:
        known = set(store[puller])
        for nm in store[peer]:
            if nm not in known:
                store[puller].append(nm)
        events[name] = (puller, head[puller], head[peer])
        order.append(name)
        store[puller].append(name)
        head[puller] = name
        txs[name] = 1
        calls[puller].append(len(store[puller]))
    return events, order, store, calls, txs
