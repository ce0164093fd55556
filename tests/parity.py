"""Shared parity helpers: run the Go-faithful oracle and the HIP engine on the
same submission stream and schedule and compare everything observable."""
import numpy as np

from babble_amd.gossip import schedule
from oracle.oracle import replay as oracle_replay


def oracle_run(dag, calls, order_seed=0):
    return oracle_replay(dag, calls, order_seed)


def compare_replay(eng, dag, calls, check_state=True, check_events=True):
    """Replay on both sides; assert identical results.  Returns (oracle, order)."""
    o, ost, oorder, ocounts = oracle_run(dag, calls)
    st, order, counts = eng.replay(dag, calls)
    # admission: ids for accepted, errors for rejected (engine adds -6 for index lies only)
    np.testing.assert_array_equal(st, ost, err_msg="admission status differs")
    assert len(order) == len(oorder), f"ordered {len(order)} vs oracle {len(oorder)}"
    np.testing.assert_array_equal(order, oorder, err_msg="consensus order differs")
    np.testing.assert_array_equal(counts, ocounts, err_msg="per-call batch sizes differ")
    if check_state:
        compare_state(eng, o, check_events)
    return o, order


def compare_state(eng, o, check_events=True):
    assert eng.rounds() == o.rounds(), (eng.rounds(), o.rounds())
    assert eng.last_consensus_round() == o.last_consensus_round()
    assert eng.last_committed_round_events() == o.last_committed_round_events()
    assert eng.consensus_transactions() == o.consensus_transactions()
    np.testing.assert_array_equal(eng.undetermined(), o.undetermined())
    np.testing.assert_array_equal(eng.consensus_events(), o.consensus_events())
    np.testing.assert_array_equal(eng.known(), o.known())
    if not check_events:
        return
    E = o.L.hgo_event_count(o.h)
    for r in range(o.rounds()):
        wits = o.round_witnesses(r)
        assert eng.round_witnesses(r) == wits, f"round {r} witnesses"
        for w in wits:
            c = eng_creator(eng, w)
            assert eng.fame(r, c) == o.round_fame(r, w), f"fame of {w} (round {r})"
    for x in range(E):
        assert eng.round(x) == o.round(x), f"round of {x}"
        assert eng.witness(x) == o.witness(x), f"witness flag of {x}"
    for x in o.consensus_events():
        assert eng.round_received(int(x)) == o.round_received(int(x)), f"rr of {x}"
        assert eng.consensus_timestamp(int(x)) == o.consensus_timestamp(int(x)), f"cts of {x}"


def eng_creator(eng, x):
    la, fd = eng.coordinates(x)
    # the creator is the column where LA == FD == own index; recover via known ids
    return _creator_cache(eng)[x]


def _creator_cache(eng):
    if not hasattr(eng, "_creators") or len(eng._creators) != eng.event_count():
        eng._creators = None
    if eng._creators is None:
        raise RuntimeError("set eng._creators before compare_state")
    return eng._creators


def with_creators(eng, dag, status):
    eng._creators = {int(s): int(c) for s, c in zip(status, dag["creator"]) if s >= 0}
    return eng


def run_case(eng, dag, k, check_events=True):
    calls = schedule(len(dag["creator"]), k)
    o, ost, oorder, ocounts = oracle_run(dag, calls)
    st, order, counts = eng.replay(dag, calls)
    with_creators(eng, dag, st)
    np.testing.assert_array_equal(st, ost, err_msg="admission status differs")
    assert len(order) == len(oorder), f"ordered {len(order)} vs oracle {len(oorder)}"
    np.testing.assert_array_equal(order, oorder, err_msg="consensus order differs")
    np.testing.assert_array_equal(counts, ocounts, err_msg="per-call batch sizes differ")
    compare_state(eng, o, check_events)
    return o, order


STREAM_KEYS = ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")


def load_golden(path):
    """(stream dict, golden npz) of a tests/golden file; streams not stored in
    the file are regenerated from its `gen` parameters (make_golden.py)."""
    from babble_amd.gossip import random_gossip
    g = np.load(path, allow_pickle=False)
    if "creator" in g.files:
        dag = {k: g[k] for k in STREAM_KEYS}
        dag["n"] = int(g["n"])
    else:
        n, events, seed, fk, fp, cp = g["gen"].tolist()
        dag = random_gossip(n, events, seed=seed, forkers=fk, fork_p=fp / 1e6, cascade_p=cp / 1e6)
    return dag, g


def compare_golden(eng, dag, g):
    """Replay `dag` on the engine and assert every field of golden `g`."""
    st, order, counts = eng.replay(dag, g["calls"])
    np.testing.assert_array_equal(st, g["status"], err_msg="admission status")
    assert len(order) == len(g["order"]), (len(order), len(g["order"]))
    np.testing.assert_array_equal(order, g["order"], err_msg="consensus order")
    np.testing.assert_array_equal(counts, g["counts"], err_msg="per-call batch sizes")
    R, lcr, lcre, ctx = g["scalars"].tolist()
    assert eng.rounds() == R
    assert eng.last_consensus_round() == (None if lcr < 0 else lcr)
    assert eng.last_committed_round_events() == lcre
    assert eng.consensus_transactions() == ctx
    np.testing.assert_array_equal(eng.undetermined(), g["undetermined"], err_msg="undetermined")
    rounds, wit = eng.event_rounds()
    np.testing.assert_array_equal(rounds, g["rounds"], err_msg="rounds")
    np.testing.assert_array_equal(wit, g["witness"].astype(bool), err_msg="witness flags")
    rr, cts = eng.event_received()
    np.testing.assert_array_equal(rr, g["rr"], err_msg="roundReceived")
    ordered = g["order"]
    np.testing.assert_array_equal(cts[ordered], g["cts"][ordered], err_msg="consensus timestamps")
    fame = g["fame"]
    for r in range(fame.shape[0]):
        for c in range(fame.shape[1]):
            if fame[r, c] >= 0:
                assert eng.fame(r, c) == fame[r, c], f"fame of round {r} creator {c}"
    return order


def s_limbs(S):
    return S.reshape(-1, 4, 8)[:, :, ::-1].copy().view("<u8").reshape(-1, 4)  # big-endian limbs


def check_run(dag, st, order, counts, rounds, wit, rr, cts):
    acc = st >= 0
    E = int(acc.sum())
    assert len(rounds) == E
    idmap = np.full(len(st) + 1, -1, np.int64)
    idmap[:-1][acc] = st[acc]
    sp = dag["sp"][acc].astype(np.int64)
    op = dag["op"][acc].astype(np.int64)
    sp_id = np.where(sp >= 0, idmap[np.maximum(sp, 0)], -1)
    op_id = np.where(op >= 0, idmap[np.maximum(op, 0)], -1)
    # the order: distinct accepted events, batches add up
    assert len(np.unique(order)) == len(order) and (order >= 0).all() and (order < E).all()
    assert counts.sum() == len(order)
    # rounds and witnesses
    has = sp_id >= 0
    pr = np.zeros(E, np.int64)
    pr[has] = np.maximum(rounds[sp_id[has]], rounds[op_id[has]])
    inc = rounds - pr
    assert ((inc == 0) | (inc == 1)).all(), "Round(x) - ParentRound(x) not in {0, 1}"
    exp_wit = ~has | (rounds > np.where(has, rounds[np.maximum(sp_id, 0)], -1))
    np.testing.assert_array_equal(wit, exp_wit, err_msg="witness = first event of its round on its chain")
    # received rounds
    ordered = np.zeros(E, bool)
    ordered[order] = True
    assert (rr[ordered] > rounds[ordered]).all(), "roundReceived must be after the event's round"
    assert (rr[~ordered] == -1).all(), "an unordered event has no roundReceived"
    # ConsensusSorter keys strictly increase inside every call's batch
    S = s_limbs(dag["S"][acc])[order]
    key_rr, key_ts = rr[order].astype(np.int64), cts[order]
    bounds = np.cumsum(counts)
    same_batch = np.ones(len(order) - 1, bool)
    same_batch[bounds[bounds < len(order)] - 1] = False
    a, b = slice(0, -1), slice(1, None)
    less = key_rr[a] < key_rr[b]
    eq = key_rr[a] == key_rr[b]
    less |= eq & (key_ts[a] < key_ts[b])
    eq &= key_ts[a] == key_ts[b]
    for limb in range(4):
        less |= eq & (S[a, limb] < S[b, limb])
        eq &= S[a, limb] == S[b, limb]
    assert (less | ~same_batch).all(), "ConsensusSorter order violated inside a batch"


def check_prefix(gp, order, counts, rounds, wit, rr, cts, fame):
    """Fields of a full replay that a committed oracle prefix golden pins
    (tests/golden/make_bench_prefix.py: the oracle on the first P submissions of
    the same stream, same schedule).  The engine reproduces per-call semantics,
    so in the full run: the first calls' batches and order equal the prefix's;
    every prefix event's round and witness flag are the prefix's (a round
    depends only on ancestors); every event the prefix ordered has the prefix's
    round received and consensus timestamp; fame of every round up to the
    prefix's LastConsensusRound is final (DecideFame restarts at LCR + 1,
    hashgraph.go:590-595).  Returns the names of the fields that differ."""
    bad = []
    nc = int(gp["n_calls"])
    if not np.array_equal(counts[:nc], gp["counts"]):
        bad.append("counts")
    go = gp["order"]
    if not np.array_equal(order[:len(go)], go):
        bad.append("order")
    if "rounds" not in gp.files:
        return bad
    P = len(gp["rounds"])
    if not np.array_equal(rounds[:P], gp["rounds"]):
        bad.append("rounds")
    if not np.array_equal(np.asarray(wit[:P]).astype(bool), gp["witness"].astype(bool)):
        bad.append("witness")
    if not np.array_equal(rr[go], gp["rr"][go]):
        bad.append("rr")
    if not np.array_equal(cts[go], gp["cts"][go]):
        bad.append("cts")
    lcr = int(gp["scalars"][1])
    if lcr >= 0 and (fame.shape[0] <= lcr or not np.array_equal(fame[:lcr + 1], gp["fame"][:lcr + 1])):
        bad.append("fame")
    return bad
