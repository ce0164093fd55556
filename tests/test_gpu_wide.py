"""Sweep coordinates at small N against the live oracle, and the wide online
path against the bulk replay (the wide goldens are in test_gpu_golden.py)."""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip
from parity import run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,events,k", [(4, 1000, 4), (16, 3000, 16), (16, 3000, 1), (32, 4000, 32),
                                        (7, 2000, 50)])
def test_sweep_coordinates_small_n(n, events, k):
    """Sweeps + transposes at small N (several sweep groups, K from 1 to 50) vs the live oracle."""
    from babble_amd.engine import Engine
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, random_gossip(n, events, seed=400 + n + k), k)
    finally:
        eng.close()


def test_wide_online_matches_replay():
    """N=64 through the online API (one batch per RunConsensus) equals the bulk replay."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import schedule
    n, E, k = 64, 3000, 64
    dag = random_gossip(n, E, seed=21)
    calls = schedule(E, k)
    a = Engine(n, 1 << 13)
    b = Engine(n, 1 << 13)
    try:
        _, order, _ = a.replay(dag, calls)
        ev = events_array(dag)
        nxt = 0
        for c in calls:
            b.insert_events(ev[nxt:c].copy())
            b.run_consensus()
            nxt = c
        np.testing.assert_array_equal(b.consensus_events(), order)
        assert b.rounds() == a.rounds()
    finally:
        a.close()
        b.close()
