"""Wide hashgraphs (N > 32) on the GPU: chain-prefix sweep coordinates, the
transposed firstDescendants runs (babble_amd/csrc/hge_coords.hip) and the
cooperative rounds kernel (hge_rounds_coop.hip), bit-exact against committed
oracle outputs (tests/golden/wide_*.npz, made by tests/golden/make_golden.py);
plus the sweep coordinates at small N against the live oracle."""
import glob
import os

import numpy as np
import pytest

from babble_amd.gossip import random_gossip
from parity import run_case

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WIDE = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "wide_*.npz")))


@pytest.mark.parametrize("path", WIDE, ids=lambda p: os.path.basename(p))
def test_wide_golden(path):
    from babble_amd.engine import Engine
    g = np.load(path, allow_pickle=False)
    n = int(g["n"])
    dag = {k: g[k] for k in ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")}
    dag["n"] = n
    eng = Engine(n, len(g["creator"]) + 16)
    try:
        st, order, counts = eng.replay(dag, g["calls"])
        np.testing.assert_array_equal(st, g["status"])
        assert len(order) == len(g["order"])
        np.testing.assert_array_equal(order, g["order"])
        np.testing.assert_array_equal(counts, g["counts"])
        R, lcr, lcre, ctx = g["scalars"].tolist()
        assert eng.rounds() == R
        assert eng.last_consensus_round() == (None if lcr < 0 else lcr)
        assert eng.last_committed_round_events() == lcre
        assert eng.consensus_transactions() == ctx
        np.testing.assert_array_equal(eng.undetermined(), g["undetermined"])
        E = len(g["rounds"])
        rounds = np.array([eng.round(x) for x in range(E)])
        np.testing.assert_array_equal(rounds, g["rounds"])
        wit = np.array([eng.witness(x) for x in range(E)])
        np.testing.assert_array_equal(wit, g["witness"])
        for x in g["order"][:: max(1, len(g["order"]) // 200)]:
            assert eng.round_received(int(x)) == int(g["rr"][x])
            assert eng.consensus_timestamp(int(x)) == int(g["cts"][x])
    finally:
        eng.close()


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
