"""Speculative parallel frontier walk (hge_walk_spec.hip) vs the oracle.

From a fresh state with long chains, DivideRounds' frontier is walked by up to
32 walkers that start from guessed frontiers and merge into each other
(k_walk_spec / k_walk_join); a walker whose history fills up without a merge
ends the chain and the sequential walk resumes there.  Every case is bit-exact
against the Go-faithful oracle (rounds, witnesses, fame, order), for several
walker counts (HGE_WALKERS), both LDS layouts (N <= 16 and 16 < N <= 32) and
the forced capacity fallback (HGE_WALK_HCAP).
"""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip
from parity import run_case

pytestmark = pytest.mark.gpu


def _run(n, events, k, seed, monkeypatch, walkers=None, hcap=None, check_events=True):
    from babble_amd.engine import Engine
    if walkers is not None:
        monkeypatch.setenv("HGE_WALKERS", str(walkers))
    if hcap is not None:
        monkeypatch.setenv("HGE_WALK_HCAP", str(hcap))
    dag = random_gossip(n, events, seed=seed)
    eng = Engine(n, 1 << 12)
    try:
        run_case(eng, dag, k, check_events=check_events)
        return eng.rounds()
    finally:
        eng.close()


def test_spec_walk_default_16_100k(monkeypatch):
    """The bench workload (16 participants, 100k events, K = 16), default walkers."""
    monkeypatch.delenv("HGE_WALKERS", raising=False)
    monkeypatch.delenv("HGE_WALK_HCAP", raising=False)
    assert _run(16, 100_000, 16, 1, monkeypatch) > 500


@pytest.mark.parametrize("walkers", [2, 3, 5, 16, 32, 64])
def test_spec_walk_walker_counts(monkeypatch, walkers):
    _run(16, 30_000, 16, 100 + walkers, monkeypatch, walkers=walkers)


@pytest.mark.parametrize("n,events,walkers", [(7, 20_000, 8), (24, 40_000, 12), (32, 60_000, 32)])
def test_spec_walk_widths(monkeypatch, n, events, walkers):
    _run(n, events, n, 200 + n, monkeypatch, walkers=walkers)


@pytest.mark.parametrize("hcap", [2, 5, 40])
def test_spec_walk_capacity_fallback(monkeypatch, hcap):
    """Histories too short to merge: the chain ends early and the sequential
    walk finishes the job from the last true row."""
    _run(16, 30_000, 16, 300 + hcap, monkeypatch, walkers=16, hcap=hcap)


def test_spec_walk_one_shot(monkeypatch):
    """One RunConsensus over the whole graph (the hashgraph_test schedule)."""
    _run(16, 30_000, 30_000, 400, monkeypatch, walkers=16)


def test_spec_walk_equals_sequential_rounds(monkeypatch):
    """Per-event rounds and witness flags from the speculative walk equal the
    sequential walk's on the same graph (HGE_WALKERS=0)."""
    from babble_amd.engine import Engine
    from babble_amd.gossip import schedule
    n, E, k = 16, 50_000, 16
    dag = random_gossip(n, E, seed=500)
    calls = schedule(E, k)
    out = []
    for w in (0, 24):
        monkeypatch.setenv("HGE_WALKERS", str(w))
        eng = Engine(n, 1 << 12)
        st, order, counts = eng.replay(dag, calls)
        ids = [int(s) for s in st if s >= 0]
        out.append((np.array([eng.round(x) for x in ids]), np.array([eng.witness(x) for x in ids]),
                    order, counts, eng.rounds()))
        eng.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
