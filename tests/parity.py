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
