"""The fresh replay at N = 256 against the engine's other paths: the online
per-call path, a replay whose rounds table overflows and grows mid-walk, and
repeated replays of the staged stream (the bench's steps).  The 256-participant
goldens (test_gpu_golden.py) and the bench's 819,200-submission prefix check the
replay against the oracle."""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule

pytestmark = pytest.mark.gpu


def _state(eng):
    _, order, counts = eng.fetch()
    return order, counts, eng.event_rounds(), eng.event_received()


def test_pipelined_replay_equals_online_path():
    """256 participants, 235 calls: the replay and the online API (one batch per
    RunConsensus) give the same order, batches, rounds and round received."""
    from babble_amd.engine import Engine, events_array
    n, E, k = 256, 60_000, 256
    dag = random_gossip(n, E, seed=77)
    ev = events_array(dag)
    calls = schedule(E, k)
    a = Engine(n, E)
    b = Engine(n, E)
    try:
        _, order, counts = a.replay(ev, calls)
        assert len(calls) >= 32 and len(order) > 0
        nxt = 0
        per = []
        for c in calls:
            b.insert_events(ev[nxt:c].copy())
            per.append(len(b.run_consensus()))
            nxt = c
        np.testing.assert_array_equal(b.consensus_events(), order)
        np.testing.assert_array_equal(np.asarray(per), counts)
        assert b.rounds() == a.rounds()
        assert b.last_consensus_round() == a.last_consensus_round()
        np.testing.assert_array_equal(b.event_rounds(), a.event_rounds())
        np.testing.assert_array_equal(b.event_received(), a.event_received())
    finally:
        a.close()
        b.close()


def test_pipelined_replay_overflow_falls_back():
    """An engine sized for a few rounds overflows its rounds table during the walk:
    it grows the table and walks again, with the same result."""
    from babble_amd.engine import Engine, events_array
    n, E, k = 256, 400_000, 256
    dag = random_gossip(n, E, seed=78)
    ev = events_array(dag)
    calls = schedule(E, k)
    small = Engine(n, 1024)
    big = Engine(n, E)
    try:
        small.replay(ev, calls)
        big.replay(ev, calls)
        for x, y in zip(_state(small), _state(big)):
            np.testing.assert_array_equal(x, y)
        assert small.rounds() == big.rounds() > 66
    finally:
        small.close()
        big.close()


def test_pipelined_replay_repeats():
    """Replaying the staged stream again (the bench's steps) gives the same state."""
    from babble_amd.engine import Engine, events_array
    n, E, k = 256, 50_000, 256
    dag = random_gossip(n, E, seed=79)
    eng = Engine(n, E)
    try:
        eng.prepare(events_array(dag), schedule(E, k))
        eng.run()
        first = _state(eng)
        for _ in range(2):
            eng.run()
            for x, y in zip(first, _state(eng)):
                np.testing.assert_array_equal(x, y)
    finally:
        eng.close()
