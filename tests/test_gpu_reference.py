"""The reference's own known-answer tests, run on the HIP engine through the C ABI.

tests/test_oracle_reference.py pins the CPU oracle to these answers; this file
asserts the same answers on the product path (hashgraph_test.go, core_test.go,
node_test.go; file:line per test).  Coordinates: the reference's
firstDescendants sentinel math.MaxInt64 (hashgraph.go:404-406) is the engine's
INT32_MAX (an unset int32 cell); lastAncestors -1 is -1 on both sides.
"""
import numpy as np
import pytest

from refdags import CONSENSUS_DAG, ROUND_DAG, SMALL_DAG, TS_BASE, fixed_bytes, playbook_views, to_stream

pytestmark = pytest.mark.gpu
INT64_MAX = np.iinfo(np.int64).max
INT32_MAX = np.iinfo(np.int32).max


def build(dag):
    from babble_amd.engine import Engine, events_array
    s, pos = to_stream(dag)
    eng = Engine(s["n"], 256)
    ids = eng.insert_events(events_array(s))
    assert ids.tolist() == list(range(len(dag)))  # engine id == insertion order
    return eng, pos


# ---- hashgraph_test.go:131-242 (initHashgraph) ----
def test_ancestor_self_ancestor_see():
    eng, ix = build(SMALL_DAG)
    A = lambda x, y: eng.ancestor(ix[x], ix[y])
    for x, y in [("e01", "e0"), ("e01", "e1"), ("e20", "e01"), ("e20", "e2"), ("e12", "e20"),
                 ("e12", "e1"), ("e20", "e0"), ("e20", "e1"), ("e12", "e01"), ("e12", "e2"),
                 ("e12", "e0"), ("e12", "e1")]:
        assert A(x, y), (x, y)
    assert not A("e01", "e2")
    S = lambda x, y: eng.self_ancestor(ix[x], ix[y])
    assert S("e01", "e0") and S("e20", "e2") and S("e12", "e1")
    for x, y in [("e01", "e1"), ("e20", "e01"), ("e12", "e20"), ("e20", "e0"), ("e12", "e2")]:
        assert not S(x, y)
    for x, y in [("e01", "e0"), ("e01", "e1"), ("e20", "e0"), ("e20", "e01"), ("e12", "e01"),
                 ("e12", "e0"), ("e12", "e1")]:
        assert eng.see(ix[x], ix[y])
    eng.close()


# ---- hashgraph_test.go:371-516 (TestInsertEvent): exact coordinates and wire info ----
def test_insert_event_coordinates():
    eng, ix = build(ROUND_DAG)
    M = INT64_MAX
    exp = {
        "e0": ([0, -1, -1], [0, 1, 1], (-1, -1, -1, 0)),
        "e21": ([0, 1, 1], [1, 2, 1], (0, 1, 1, 2)),
        "f1": ([1, 2, 1], [M, 2, M], (1, 0, 1, 1)),
    }
    for name, (la, fd, wire) in exp.items():
        gla, gfd = eng.coordinates(ix[name])
        gfd = [M if v == INT32_MAX else int(v) for v in gfd]
        assert gla.tolist() == la, name
        assert gfd == fd, name
        assert eng.wire_info(ix[name]) == wire, name
    eng.close()


# ---- hashgraph_test.go:563-612 ----
def test_strongly_see():
    eng, ix = build(ROUND_DAG)
    SS = lambda x, y: eng.strongly_see(ix[x], ix[y])
    for x, y in [("e21", "e0"), ("e02", "e10"), ("e02", "e0"), ("e02", "e1"), ("f1", "e21"),
                 ("f1", "e10"), ("f1", "e0"), ("f1", "e1"), ("f1", "e2")]:
        assert SS(x, y), (x, y)
    for x, y in [("e10", "e0"), ("e21", "e1"), ("e21", "e2"), ("e02", "e2"), ("f1", "e02")]:
        assert not SS(x, y), (x, y)
    eng.close()


# ---- hashgraph_test.go:614-742: rounds with Store.SetRound in place of DivideRounds ----
def test_parent_round_witness_round_inc_round_diff():
    eng, ix = build(ROUND_DAG)
    eng.set_round(0, [(ix["e0"], True, 0), (ix["e1"], True, 0), (ix["e2"], True, 0)])
    assert eng.rounds() == 1
    assert eng.round_inc(ix["f1"])                   # TestRoundInc
    assert not eng.round_inc(ix["e02"])
    assert eng.round(ix["f1"]) == 1                  # TestRound
    assert eng.round(ix["e02"]) == 0
    assert eng.round_diff(ix["f1"], ix["e02"]) == 1  # TestRoundDiff
    assert eng.round_diff(ix["e02"], ix["f1"]) == -1
    assert eng.round_diff(ix["e02"], ix["e21"]) == 0
    eng.set_round(1, [(ix["f1"], True, 0)])
    assert eng.rounds() == 2
    for nm in ("e0", "e1", "e10", "f1"):             # TestParentRound
        assert eng.parent_round(ix[nm]) == 0, nm
    for nm in ("e0", "e1", "e2", "f1"):              # TestWitness
        assert eng.witness(ix[nm]), nm
    for nm in ("e10", "e21", "e02"):
        assert not eng.witness(ix[nm]), nm
    assert eng.parent_round(len(ROUND_DAG)) == -1    # unknown event
    eng.close()


def test_divide_rounds():
    eng, ix = build(ROUND_DAG)
    eng.divide_rounds()
    assert eng.rounds() == 2
    assert eng.round_witnesses(0) == sorted([ix["e0"], ix["e1"], ix["e2"]])
    assert eng.round_witnesses(1) == [ix["f1"]]
    eng.close()


# ---- hashgraph_test.go:952-1070 (initConsensusHashgraph) ----
def test_decide_fame_round_received_find_order_known():
    eng, ix = build(CONSENSUS_DAG)
    assert eng.oldest_self_ancestor_to_see(ix["f0"], ix["e1"]) == ix["e02"]
    assert eng.oldest_self_ancestor_to_see(ix["f1"], ix["e0"]) == ix["e10"]
    assert eng.oldest_self_ancestor_to_see(ix["e21"], ix["e1"]) == ix["e21"]
    assert eng.oldest_self_ancestor_to_see(ix["e2"], ix["e1"]) is None
    eng.divide_rounds()
    eng.decide_fame()
    for nm in ("g0", "g1", "g2"):
        assert eng.round(ix[nm]) == 2
    for c in range(3):
        assert eng.fame(0, c) == 1  # e0, e1, e2 famous
    eng.decide_round_received()
    for nm, i in ix.items():
        if nm.startswith("e"):
            assert eng.round_received(i) == 1, nm
    order = eng.find_order()
    names = {v: k for k, v in ix.items()}
    got = [names[int(i)] for i in order]
    exp1 = ["e0", "e10", "e1", "e21", "e2", "e02"]
    exp2 = ["e0", "e1", "e10", "e2", "e21", "e02"]
    assert len(got) == 6 and all(g in (exp1[i], exp2[i]) for i, g in enumerate(got))
    assert got == ["e0", "e1", "e10", "e2", "e21", "e02"]  # exact for the fixture's S bytes
    assert eng.known().tolist() == [7, 7, 7]
    eng.close()


# ---- node/core_test.go:339-387, node/node_test.go:279-391 ----
def test_consensus_playbook_three_cores():
    from babble_amd.engine import Engine
    events, order, store, calls, txs = playbook_views()
    res = []
    for core in range(3):
        eng = Engine(3, 256)
        ids, seq = {}, {}
        for k, nm in enumerate(store[core]):
            c, sp, op = events[nm]
            idx = seq.get(c, 0)
            seq[c] = idx + 1
            ids[nm] = eng.insert(c, idx, ids[sp] if sp else -1, ids[op] if op else -1,
                                 TS_BASE + 1000 * order.index(nm), fixed_bytes(nm, "S"),
                                 fixed_bytes(nm, "H"), txs.get(nm, 0))
            if (k + 1) in calls[core]:
                eng.run_consensus()
        names = {v: k for k, v in ids.items()}
        res.append((eng, [names[int(i)] for i in eng.consensus_events()]))
    assert len(res[0][1]) == 6
    assert res[0][1] == res[1][1] == res[2][1]        # TestConsensus
    e0 = res[0][0]
    assert e0.last_consensus_round() == 1              # TestStats
    assert e0.consensus_transactions() == 3
    assert len(e0.undetermined()) == 14
    for eng, o in res:                                 # TestTransactionOrdering
        assert [nm for nm in o if nm in ("e10", "e21", "e02")] == ["e10", "e21", "e02"]
        eng.close()


# ---- hashgraph.go:366-396 FromParentsLatest on the engine ----
def test_fork_rejection_codes():
    from babble_amd.engine import HgeError
    eng, ix = build(ROUND_DAG)
    cases = [((1, 1, ix["e1"], ix["e0"]), -5),   # second child of e1: fork
             ((2, 2, ix["e21"], 999), -4),        # unknown other-parent
             ((0, 0, -1, -1), -2),                # second initial event of creator 0
             ((0, 2, ix["e10"], ix["e21"]), -3),  # self-parent by another creator
             ((7, 0, -1, -1), -1)]                # unknown creator
    for (c, idx, sp, op), code in cases:
        with pytest.raises(HgeError) as ei:
            eng.insert(c, idx, sp, op, TS_BASE)
        assert ei.value.code == code, (c, idx, sp, op)
    assert eng.event_count() == len(ROUND_DAG)  # nothing was inserted
    eng.close()


def test_index_lying_event_is_a_documented_deviation():
    """The reference accepts an event whose Body.Index is not its chain position
    (FromParentsLatest never looks at it, hashgraph.go:366-396); the engine refuses
    it with HGE_ERR_INDEX (include/hge.h): its tables are indexed
    by chain position.  Honest events are unaffected."""
    from babble_amd.engine import HgeError
    from oracle.oracle import Oracle
    eng, ix = build(ROUND_DAG)
    with pytest.raises(HgeError) as ei:
        eng.insert(2, 5, ix["e21"], ix["f1"], TS_BASE + 10**6)  # e21 is index 1: next is 2
    assert ei.value.code == -6
    o = Oracle(3)
    s, _ = to_stream(ROUND_DAG)
    for i in range(len(ROUND_DAG)):
        o.insert(int(s["creator"][i]), int(s["index"][i]), int(s["sp"][i]), int(s["op"][i]), int(s["ts"][i]))
    assert o.insert(2, 5, ix["e21"], ix["f1"], TS_BASE + 10**6) == len(ROUND_DAG)  # accepted there
    eng.insert(2, 2, ix["e21"], ix["f1"], TS_BASE + 10**6)  # the honest index goes in
    eng.close()


def test_insert_batch_error_carries_accepted_ids():
    from babble_amd.engine import Engine, HgeError, events_array
    s, ix = to_stream(ROUND_DAG)
    ev = events_array(s)
    bad = ev[3:4].copy()
    bad["self_parent"] = 999
    eng = Engine(3, 256)
    with pytest.raises(HgeError) as ei:
        eng.insert_events(np.concatenate([ev[:3], bad, ev[4:]]))
    assert ei.value.code == -2
    assert ei.value.accepted.tolist() == [0, 1, 2]
    assert eng.event_count() == 3
    eng.close()


def test_cpp_abi_binary_on_gpu():
    """tests/abi/hge_abi_test.cpp --gpu: the consensus DAG through the C ABI from C++."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([os.path.join(root, "build", "hge_abi_test"), "--gpu"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr + out.stdout


def test_go_shim_logic_replayed_on_gpu():
    """tests/abi/shim_replay_test.cpp --gpu: the Go shim's Hashgraph + bound InmemStore
    restated in C++ (hash <-> id map, tsByNano, FindOrder's batch mapping) through
    TestFindOrder, and a SetRound before consensus that GetRound must not let hide the
    fame the engine decides afterwards."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([os.path.join(root, "build", "shim_replay_test"), "--gpu"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr + out.stdout
    assert "0 failures" in out.stdout


@pytest.mark.parametrize("n,events,k", [(4, 800, 4), (16, 3000, 16), (64, 4000, 64)])
def test_consensus_timestamp_sources(n, events, k):
    """hge_consensus_timestamp_sources (MedianTimestamp's source, hashgraph.go:762-770):
    every ordered event's source has the consensus timestamp as its own timestamp and is
    OldestSelfAncestorToSee(w, x) of a famous witness w of x's round received that sees
    x (the oracle's predicates); unordered events have none."""
    from babble_amd.engine import Engine
    from babble_amd.gossip import random_gossip, schedule
    from oracle.oracle import replay as oracle_replay
    # timestamps with repeats: several candidates share an instant
    dag = random_gossip(n, events, seed=61)
    dag["ts"] = dag["ts"] // 7000 * 7000
    calls = schedule(events, k)
    eng = Engine(n, events + 64)
    try:
        st, order, _ = eng.replay(dag, calls)
        o, ost, oorder, _ = oracle_replay(dag, calls)
        assert np.array_equal(order, oorder)
        ids = np.arange(len(st), dtype=np.int32)
        src = eng.consensus_timestamp_sources(ids)
        rr, cts = eng.event_received()
        assert (st == np.arange(len(st))).all()  # no forks: engine id = submission index
        ts = dag["ts"]
        assert (src[rr < 0] == -1).all()
        ordered = set(order.tolist())
        assert ordered == set(np.nonzero(rr >= 0)[0].tolist())
        for x in list(ordered)[:400]:
            s = int(src[x])
            assert s >= 0 and ts[s] == cts[x]
            cands = set()
            for w in o.round_witnesses(int(rr[x])):
                if o.round_fame(int(rr[x]), w) == 1 and o.see(w, x):
                    cands.add(o.oldest_self_ancestor_to_see(w, x))
            assert s in cands
    finally:
        eng.close()
